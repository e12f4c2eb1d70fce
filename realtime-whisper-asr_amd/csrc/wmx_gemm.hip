// MFMA GEMM  C[M,N] = A[M,K] . W[N,K]^T  with fused epilogues (SURVEY.md §2a "GEMM", "Conv1D", "Logits").
//
// Both operands are K-contiguous 16-bit (bf16 or f16) so A and W tiles share one LDS image and one fragment
// read.  Tiles are staged HBM -> LDS with global_load_lds_dwordx4 (lane-linear 1 KiB per wave instruction);
// the bank-conflict XOR swizzle (16-B piece ^= row & 7) is applied on the global SOURCE address and on the
// ds_read, never on the LDS destination (cdna_hip_programming.md §5.4 rule 21).  Two LDS buffers, BK = 64,
// v_mfma_f32_16x16x32_{bf16,f16}, fp32 accumulation.  Block index is XCD-remapped so consecutive N tiles of
// one row panel share an XCD's L2 (§5.5 T1, bijective form).
//
// Epilogues are fused: bias, exact-erf GELU, fp32 residual add (the residual stream stays fp32), conv2's
// GELU + sinusoidal position add, the decoder QKV scatter straight into the self-attention KV cache, and
// split-K fp32 partial slabs reduced deterministically (fixed order) by gemm_splitk_reduce.
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "wmx_common.h"
#include "wmx_kernels.h"

#include <type_traits>

namespace wmx {

// K and V^T of [L][xw][H] (window, head) images, each kXS x 64 in the fragment-major order of crossk_off /
// crossv_off (wmx_kernels.h): each (window, head) is one contiguous stream for the decode step, read as whole
// 1 KiB pieces that are already the MFMA operands of S^T = K.Q^T and P.V
__device__ inline long crosskv_index(const Epi& e, int m, int n) {
  const int w = m / e.xt, t = m - w * e.xt;
  const int lk = n / e.d, c = n - lk * e.d;
  const long base = (((long)lk * e.xw + w) * (e.d >> 6) + (c >> 6)) * 64 * kXS;
  return base + ((lk & 1) ? crossv_off(t, c & 63) : crossk_off(t, c & 63));
}

template <DT T>
__device__ inline void epi_store(const Epi& e, int m, int n, float v) {
  if (e.bias) v += e.bias[n];
  switch (e.kind) {
    case EPI_STORE16:
      reinterpret_cast<uint16_t*>(e.out)[(long)m * e.ldc + n] = from_f32<T>(v);
      break;
    case EPI_GELU16:
      reinterpret_cast<uint16_t*>(e.out)[(long)m * e.ldc + n] = from_f32<T>(gelu_erf(v));
      break;
    case EPI_RESID32: {
      float* o = reinterpret_cast<float*>(e.out) + (long)m * e.ldc + n;
      *o = *o + v;
      break;
    }
    case EPI_GELU_POS32:
      reinterpret_cast<float*>(e.out)[(long)m * e.ldc + n] = gelu_erf(v) + e.pos[(long)(m % e.posT) * e.ldc + n];
      break;
    case EPI_STORE32:
      reinterpret_cast<float*>(e.out)[(long)m * e.ldc + n] = v;
      break;
    case EPI_QKV_CACHE: {
      // m = row * Tn + i ; slot = *slot0 + i ; cols [0,d) q, [d,2d) k -> cache, [2d,3d) v -> cache
      const int d = e.d;
      const uint16_t h = from_f32<T>(v);
      if (n < d) {
        reinterpret_cast<uint16_t*>(e.out)[(long)m * d + n] = h;
      } else {
        const int r = m / e.Tn, i = m - r * e.Tn;
        const long slot = (long)(*e.slot0) + i;
        uint16_t* cache = n < 2 * d ? e.kc : e.vc;
        cache[(slot * e.R + (long)r * e.rmul) * d + (n % d)] = h;
      }
      break;
    }
    case EPI_CROSSKV:
      reinterpret_cast<uint16_t*>(e.out)[crosskv_index(e, m, n)] = from_f32<T>(v);
      break;
    default:
      break;
  }
}

// four consecutive columns n..n+3 (n % 4 == 0, n + 3 < N): vectorised loads / stores
template <DT T>
__device__ inline void epi_store4(const Epi& e, int m, int n, float4 v) {
  if (e.bias) {
    const float4 b = *reinterpret_cast<const float4*>(e.bias + n);
    v.x += b.x;
    v.y += b.y;
    v.z += b.z;
    v.w += b.w;
  }
  switch (e.kind) {
    case EPI_GELU16:
      v = make_float4(gelu_erf(v.x), gelu_erf(v.y), gelu_erf(v.z), gelu_erf(v.w));
      [[fallthrough]];
    case EPI_STORE16: {
      u16x4 h = {from_f32<T>(v.x), from_f32<T>(v.y), from_f32<T>(v.z), from_f32<T>(v.w)};
      *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + (long)m * e.ldc + n) = h;
      break;
    }
    case EPI_RESID32: {
      float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(e.out) + (long)m * e.ldc + n);
      float4 x = *o;
      *o = make_float4(x.x + v.x, x.y + v.y, x.z + v.z, x.w + v.w);
      break;
    }
    case EPI_GELU_POS32: {
      const float4 p = *reinterpret_cast<const float4*>(e.pos + (long)(m % e.posT) * e.ldc + n);
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(e.out) + (long)m * e.ldc + n) =
          make_float4(gelu_erf(v.x) + p.x, gelu_erf(v.y) + p.y, gelu_erf(v.z) + p.z, gelu_erf(v.w) + p.w);
      break;
    }
    case EPI_STORE32:
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(e.out) + (long)m * e.ldc + n) = v;
      break;
    case EPI_QKV_CACHE: {
      const int d = e.d;
      u16x4 h = {from_f32<T>(v.x), from_f32<T>(v.y), from_f32<T>(v.z), from_f32<T>(v.w)};
      uint16_t* dst;
      if (n < d) {
        dst = reinterpret_cast<uint16_t*>(e.out) + (long)m * d + n;
      } else {
        const int r = m / e.Tn, i = m - r * e.Tn;
        const long slot = (long)(*e.slot0) + i;
        uint16_t* cache = n < 2 * d ? e.kc : e.vc;
        dst = cache + (slot * e.R + (long)r * e.rmul) * d + (n % d);
      }
      *reinterpret_cast<u16x4*>(dst) = h;
      break;
    }
    case EPI_CROSSKV: {
      uint16_t* o = reinterpret_cast<uint16_t*>(e.out);
      if (((n / e.d) & 1) == 0) {
        u16x4 h = {from_f32<T>(v.x), from_f32<T>(v.y), from_f32<T>(v.z), from_f32<T>(v.w)};
        *reinterpret_cast<u16x4*>(o + crosskv_index(e, m, n)) = h;
      } else {  // V^T: the 4 columns are 4 rows of the transposed image
        o[crosskv_index(e, m, n)] = from_f32<T>(v.x);
        o[crosskv_index(e, m, n + 1)] = from_f32<T>(v.y);
        o[crosskv_index(e, m, n + 2)] = from_f32<T>(v.z);
        o[crosskv_index(e, m, n + 3)] = from_f32<T>(v.w);
      }
      break;
    }
    default:
      break;
  }
}

template <DT T, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM* WN * 64) void gemm_kernel(const uint16_t* __restrict__ A, long lda,
                                                           const uint16_t* __restrict__ W, long ldw, int M, int N,
                                                           int K, int kchunk, Epi e, float* __restrict__ ws) {
  constexpr int NW = WM * WN;
  constexpr int A_CH = BM / 8, B_CH = BN / 8;  // 1 KiB chunks (8 rows x 64 k) per tile
  static_assert(A_CH % NW == 0 && B_CH % NW == 0, "tile/wave mismatch");
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int TILE_BYTES = (BM + BN) * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tilesN = (N + BN - 1) / BN;
  const int tilesM = (M + BM - 1) / BM;
  const int nwg = tilesN * tilesM;
  // bijective XCD remap: blocks b and b+8 share an XCD; give each XCD a contiguous range of tiles
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tm = bid / tilesN, tn = bid - tm * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = blockIdx.y * kchunk;
  const int ke = min(K, kb + kchunk);
  const int nk = (ke - kb) / 64;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;

  // per-lane staging source offsets (row and swizzled piece are loop-invariant)
  const int srow = lane >> 3;
  auto issue = [&](int kt, int buf) {
    char* base = smem + buf * TILE_BYTES;
    const int k0 = kb + kt * 64;
#pragma unroll
    for (int c = wave; c < A_CH; c += NW) {
      const int row = c * 8 + srow;
      const int gp = (lane & 7) ^ (row & 7);
      const int gr = min(m0 + row, M - 1);
      const uint16_t* src = A + (long)gr * lda + k0 + gp * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(base + c * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int c = wave; c < B_CH; c += NW) {
      const int row = c * 8 + srow;
      const int gp = (lane & 7) ^ (row & 7);
      const int gr = min(n0 + row, N - 1);
      const uint16_t* src = W + (long)gr * ldw + k0 + gp * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(base + BM * 128 + c * 1024), 16, 0,
                                       0);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  if (nk > 0) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, buf ^ 1);
    const char* As = smem + buf * TILE_BYTES;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int p = s * 4 + fq;
      u16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + fr;
        af[i] = *reinterpret_cast<const u16x8*>(As + row * 128 + ((p ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * (BN / WN) + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const u16x8*>(Bs + row * 128 + ((p ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16<T>(af[i], bfr[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue through LDS, WM row rounds: the waves of row group `rd` park their fp32 accumulators in a
  // [BM/WM][BN+4] image, then all threads apply the epilogue 4 columns at a time with vector stores.
  constexpr int RR = BM / WM, LDT = BN + 4;
  static_assert(RR * LDT * 4 <= 2 * TILE_BYTES, "epilogue image exceeds the staging LDS");
  float* img = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int rd = 0; rd < WM; ++rd) {
    if (wm == rd) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) img[(i * 16 + fq * 4 + r) * LDT + wn * (BN / WN) + j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    if (e.kind == EPI_CROSSKV && !ws && ((n0 / e.d) & 1)) {
      // V^T tile (the host checks d % BN == 0, xt % 4 == 0): 4 consecutive keys of one column per 8-byte store
      for (int idx = tid; idx < RR / 4 * BN; idx += NW * 64) {
        const int col = idx % BN, r4 = (idx / BN) * 4;
        const int m = m0 + rd * RR + r4, n = n0 + col;
        if (m >= M || n >= N) continue;
        const float b = e.bias ? e.bias[n] : 0.f;
        u16x4 h;
#pragma unroll
        for (int q = 0; q < 4; ++q) h[q] = from_f32<T>(img[(r4 + q) * LDT + col] + b);
        *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + crosskv_index(e, m, n)) = h;
      }
      __syncthreads();
      continue;
    }
    for (int idx = tid; idx < RR * BN / 4; idx += NW * 64) {
      const int row = idx / (BN / 4), c4 = (idx % (BN / 4)) * 4;
      const int m = m0 + rd * RR + row, n = n0 + c4;
      if (m >= M || n >= N) continue;
      const float4 v = *reinterpret_cast<const float4*>(img + row * LDT + c4);
      if (ws) {
        float* w = ws + ((long)blockIdx.y * M + m) * N + n;
        if (n + 3 < N && (N & 3) == 0) {
          *reinterpret_cast<float4*>(w) = v;
        } else {
          const float vv[4] = {v.x, v.y, v.z, v.w};
          for (int q = 0; q < 4 && n + q < N; ++q) w[q] = vv[q];
        }
      } else if (n + 3 < N && (e.ldc & 3) == 0) {
        epi_store4<T>(e, m, n, v);
      } else {
        const float vv[4] = {v.x, v.y, v.z, v.w};
        for (int q = 0; q < 4 && n + q < N; ++q) epi_store<T>(e, m, n + q, vv[q]);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// Large-M GEMM (encoder projections, conv front end, cross-K/V): 256 x 256 tile, 8 waves (2 M x 4 N, wave tile
// 128 x 64 = 8 x 4 MFMA fragments), K staged in 64-deep K-tiles (whole 128-B lines per row) through a half-tile LDS
// ring filled by global_load_lds_dwordx4 (the layout and schedule at the ring below).  Each K-tile is waited for with
// a COUNTED vmcnt (cdna_hip_programming.md §5 "Pipelining across barriers"), never vmcnt(0) in steady state and never
// __syncthreads() inside the loop.  All LDS is one extern array (§5 item 4(a)).  Against the 32-deep slice ring of
// rounds 2-4 (every 128-B line fetched in two halves one slice apart) TCP -> L2 read requests halve (qkv 13.8 M ->
// 7.2 M per launch) and the main loop takes 23 % fewer clocks (profiles/r05h_g256_k64/).
// Measured and removed in round 6: C^T fragments for the direct epilogues, unit 1 staged one phase
// later, 8 row panels per XCD group, one 32-MFMA segment per slice, per-segment s_setprio.
// ------------------------------------------------------------------------------------------------
#define WMX_G256_MFMA(a, b, c) mfma16<T>(a, b, c)
// a scheduling barrier after each segment's opening s_barrier (without it the compiler hoists the segment's first
// MFMA above the barrier, into the partner's compute segment)
#define WMX_G256_PIN __builtin_amdgcn_sched_barrier(0)
constexpr int kG256Slot = (256 + 256) * 64;  // 32 KiB
// 128 KiB ring + the LayerNorm-folded kinds' raw row statistics [8 groups][256 rows] float2 and merged (mean, rstd)
constexpr int kG256StatRaw = 4 * kG256Slot, kG256StatRow = kG256StatRaw + 8 * 256 * 8;
constexpr int kG256Lds = kG256StatRow + 256 * 8;
template <int KIND>
constexpr bool g256_lnf() { return KIND == EPI_LNF_STORE16 || KIND == EPI_LNF_GELU16; }
template <int KIND>
constexpr int g256_lds() { return g256_lnf<KIND>() ? kG256Lds : 4 * kG256Slot; }
static_assert(kG256Lds <= 163840, "gemm256 LDS");

// apply the epilogue to `rows` rows of an fp32 LDS image [rows][ldt] holding output rows mb.. and columns n0..n0+BN
template <DT T, int BN, int NT>
__device__ inline void epi_from_image(const Epi& e, const float* img, int ldt, int rows, int mb, int n0, int M, int N,
                                      int tid) {
  if (e.kind == EPI_CROSSKV && ((n0 / e.d) & 1)) {
    // V^T tile (the host checks d % BN == 0, xt % 4 == 0): 4 consecutive keys of one column per 8-byte store
    for (int idx = tid; idx < rows / 4 * BN; idx += NT) {
      const int col = idx % BN, r4 = (idx / BN) * 4;
      const int m = mb + r4, n = n0 + col;
      if (m >= M || n >= N) continue;
      const float b = e.bias ? e.bias[n] : 0.f;
      u16x4 h;
#pragma unroll
      for (int q = 0; q < 4; ++q) h[q] = from_f32<T>(img[(r4 + q) * ldt + col] + b);
      *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + crosskv_index(e, m, n)) = h;
    }
    return;
  }
  for (int idx = tid; idx < rows * BN / 4; idx += NT) {
    const int row = idx / (BN / 4), c4 = (idx % (BN / 4)) * 4;
    const int m = mb + row, n = n0 + c4;
    if (m >= M || n >= N) continue;
    const float4 v = *reinterpret_cast<const float4*>(img + row * ldt + c4);
    if (n + 3 < N && (e.ldc & 3) == 0) {
      epi_store4<T>(e, m, n, v);
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int q = 0; q < 4 && n + q < N; ++q) epi_store<T>(e, m, n + q, vv[q]);
    }
  }
}

// fast form of epi_from_image for a 64-row x 256-column image and 512 threads: a thread owns one column quad
// and rows r0, r0 + 8, ... (r0 = tid / 64): the bias is loaded once, and every row's loads (image, residual,
// position) are issued before its stores, so the store tail is not a chain of dependent global round trips.
// the residual rows of one 64-row epilogue round of the 256-column image (thread: column quad (tid & 63), rows
// (tid >> 6) + 8u), loaded one round ahead so the RMW epilogues (fp32 / hi-lo residual) do not wait one memory
// round trip per round; rows past M are clamped (their results are not stored)
struct Resid8 {
  float4 f[8];
  u16x4 h[8], l[8];
};
template <int KIND>
__device__ inline void resid_load(Resid8& R, const Epi& e, int mb, int n0, int M, int tid) {
  const int n = n0 + (tid & 63) * 4, r0 = tid >> 6;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const long mm = min(mb + r0 + 8 * u, M - 1);
    if (KIND == EPI_RESID32) {
      R.f[u] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(e.out) + mm * e.ldc + n);
    } else {
      R.h[u] = *reinterpret_cast<const u16x4*>(e.out16 + mm * e.ldc + n);
      R.l[u] = *reinterpret_cast<const u16x4*>(reinterpret_cast<const uint16_t*>(e.out) + mm * e.ldc + n);
    }
  }
}

// UB: rows per batch of loads (8: all of the thread's rows at once; 4: two batches, for a caller whose accumulators
// leave no room for 64 more VGPRs)
template <DT T, int KIND, int UB = 8>
__device__ inline void epi_rows64(const Epi& e, const float* img, int ldt, int mb, int n0, int M, int N, int tid,
                                  const float4* bpre = nullptr, const Resid8* pre = nullptr) {
  constexpr int KD = KIND;
  const int c4 = (tid & 63) * 4, r0 = tid >> 6;
  const int n = n0 + c4;
  if (n >= N) return;
  float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bpre)  // loaded by the caller at tile start, so no round of the epilogue waits on it
    b = *bpre;
  else if (e.bias)
    b = *reinterpret_cast<const float4*>(e.bias + n);
#pragma unroll
  for (int ub = 0; ub < 8; ub += UB) {
  float4 v[UB], aux[UB];
#pragma unroll
  for (int uu = 0; uu < UB; ++uu) {
    const int u = ub + uu;
    const int row = r0 + 8 * u, m = mb + row;
    v[uu] = *reinterpret_cast<const float4*>(img + row * ldt + c4);
    v[uu] = make_float4(v[uu].x + b.x, v[uu].y + b.y, v[uu].z + b.z, v[uu].w + b.w);
    if (KD == EPI_RESID32 && pre)
      aux[uu] = pre->f[u];
    else if (KD == EPI_RESID32 && m < M)
      aux[uu] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(e.out) + (long)m * e.ldc + n);
    if (KD == EPI_GELU_POS32 && m < M)
      aux[uu] = *reinterpret_cast<const float4*>(e.pos + (long)(m % e.posT) * e.ldc + n);
  }
#pragma unroll
  for (int uu = 0; uu < UB; ++uu) {
    const int u = ub + uu;
    const int m = mb + r0 + 8 * u;
    if (m >= M) continue;
    float4 x = v[uu];
    if (KD == EPI_GELU16 || KD == EPI_GELU_POS32 || KD == EPI_GELU_MX8) x = gelu_erf4(x);
    if (KD == EPI_RESID32 || KD == EPI_GELU_POS32)
      x = make_float4(x.x + aux[uu].x, x.y + aux[uu].y, x.z + aux[uu].z, x.w + aux[uu].w);
    if (KD == EPI_GELU_MX8) {
      // the 8 lanes of a 32-column block (c4 = 4 * (tid & 63)) agree on the block scale; every lane of the wave
      // is on the same row, so the shuffles never cross an inactive lane
      const int ex = mx8_exp(max8_lanes(fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)))));
      const float is = mx8_inv_scale(ex);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(e.out) + (long)m * e.ldc + n) =
          mx8_pack4(x.x * is, x.y * is, x.z * is, x.w * is);
      if ((tid & 7) == 0) e.out2[(long)m * e.ldc2 + (n >> 5)] = (uint8_t)(ex + 127);
    } else if (KD == EPI_STORE16 || KD == EPI_GELU16 || KD == EPI_CROSSKV) {
      const u16x4 h = {from_f32<T>(x.x), from_f32<T>(x.y), from_f32<T>(x.z), from_f32<T>(x.w)};
      uint16_t* dst = KD == EPI_CROSSKV ? reinterpret_cast<uint16_t*>(e.out) + crosskv_index(e, m, n)
                                        : reinterpret_cast<uint16_t*>(e.out) + (long)m * e.ldc + n;
      *reinterpret_cast<u16x4*>(dst) = h;
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(e.out) + (long)m * e.ldc + n) = x;
    }
  }
  }
}

// eight per-lane values v[u] (u = row of the wave's 8) -> the sum over the wave's 64 lanes of row (lane >> 3), in
// every lane of that row's 8-lane group: permlane32 / permlane16 swaps halve the rows a lane carries (4 + 2 swaps),
// a row_ror:8 exchange picks one, and an 8-lane DPP sum finishes (10 cross-lane steps instead of 8 wave sums' 48)
__device__ inline float rows8_sum(const float (&v)[8], int lane) {
  float w[4], w2[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // lanes < 32: rows j, lanes >= 32: rows j + 4, each summed over l and l ^ 32
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + 4]), false, false);
    w[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {  // 16-lane rows with bit 4 clear keep j, set keep j + 2, summed over l ^ 16
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[j]), __float_as_uint(w[j + 2]), false, false);
    w2[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool b3 = (lane >> 3) & 1;  // bit 3 keeps w2[1]
  const float keep = b3 ? w2[1] : w2[0], send = b3 ? w2[0] : w2[1];
  return sum8_lanes(keep + dpp_mov<kDppXor8>(send));
}

// LayerNorm-statistics producers of the encoder fold (host: N % 256 == 0): a 64-row x 256-column LDS image, thread =
// column quad (tid & 63) of rows r0 + 8u (r0 = wave).  x = acc + bias + hi + lo (RESID) or gelu(acc + bias) + pos
// (conv2); x is stored back as the 16-bit planes hi = 16-bit(x) (e.out16, the A operand of the LayerNorm-folded
// projection that follows) and lo = 16-bit(x - hi) (e.out), the same bytes as the fp32 row; per row, this tile's
// (mean, M2) over its 256 columns goes to stats[n0 / 256][m] (Chan's pairwise form; two rows8_sum passes).
template <DT T, int KIND>
__device__ inline void epi_rows64_lns(const Epi& e, const float* img, int ldt, int mb, int n0, int M, int tid,
                                      const float4* bpre, const Resid8* pre) {
  const int lane = tid & 63, c4 = lane * 4, r0 = tid >> 6;
  const int n = n0 + c4;
  const float4 b = *bpre;
  uint16_t* hi = e.out16;
  uint16_t* lo = reinterpret_cast<uint16_t*>(e.out);
  float4 x[8];
  u16x4 ah[8], al[8];
  float4 pp[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int row = r0 + 8 * u, mm = min(mb + row, M - 1);
    x[u] = *reinterpret_cast<const float4*>(img + row * ldt + c4);
    x[u] = make_float4(x[u].x + b.x, x[u].y + b.y, x[u].z + b.z, x[u].w + b.w);
    if (KIND == EPI_RESID32_LNS) {
      ah[u] = pre->h[u];
      al[u] = pre->l[u];
    } else {
      pp[u] = *reinterpret_cast<const float4*>(e.pos + (long)(mm % e.posT) * e.ldc + n);
    }
  }
  float s[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = mb + r0 + 8 * u;
    float4 v = x[u];
    if (KIND == EPI_RESID32_LNS) {
      v.x += to_f32<T>(ah[u][0]) + to_f32<T>(al[u][0]);
      v.y += to_f32<T>(ah[u][1]) + to_f32<T>(al[u][1]);
      v.z += to_f32<T>(ah[u][2]) + to_f32<T>(al[u][2]);
      v.w += to_f32<T>(ah[u][3]) + to_f32<T>(al[u][3]);
    } else {
      v = gelu_erf4(v);
      v = make_float4(v.x + pp[u].x, v.y + pp[u].y, v.z + pp[u].z, v.w + pp[u].w);
    }
    x[u] = v;
    const u16x4 h = {from_f32<T>(v.x), from_f32<T>(v.y), from_f32<T>(v.z), from_f32<T>(v.w)};
    const u16x4 l = {from_f32<T>(v.x - to_f32<T>(h[0])), from_f32<T>(v.y - to_f32<T>(h[1])),
                     from_f32<T>(v.z - to_f32<T>(h[2])), from_f32<T>(v.w - to_f32<T>(h[3]))};
    if (m < M) {  // uniform over the wave (one row)
      *reinterpret_cast<u16x4*>(hi + (long)m * e.ldc + n) = h;
      *reinterpret_cast<u16x4*>(lo + (long)m * e.ldc + n) = l;
    }
    s[u] = (v.x + v.y) + (v.z + v.w);
  }
  const float mean_own = rows8_sum(s, lane) * (1.0f / 256.0f);  // the mean of row (lane >> 3)
  float q[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float mean_u = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mean_own), 8 * u));
    const float a = x[u].x - mean_u, bb = x[u].y - mean_u, cc = x[u].z - mean_u, dd = x[u].w - mean_u;
    q[u] = (a * a + bb * bb) + (cc * cc + dd * dd);
  }
  const float m2 = rows8_sum(q, lane);
  const int m = mb + r0 + 8 * (lane >> 3);
  if ((lane & 7) == 0 && m < M) e.stats[(long)(n0 >> 8) * e.stats_ld + m] = make_float2(mean_own, m2);
}

// GELU -> MX-fp8 epilogue for a 64-row x 256-column image with one MX block per thread: wave w takes the 32-column
// block w and lane l row l, so the block's amax is thread-local (no lane shuffles), the 32 e4m3 bytes leave as two
// 16-byte stores and the bias of the block is wave-uniform; row r's 16-B reads sit at bank 4r (row stride 260 floats),
// conflict-free for ds_read_b128's lane groups.  Same arithmetic per element as the quad form in epi_rows64.
template <DT T>
__device__ inline void epi_gelu_mx8_blocks(const Epi& e, const float* img, int ldt, int mb, int n0, int M, int tid) {
  const int lane = tid & 63, blk = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = mb + lane, n = n0 + 32 * blk;
  const float* src = img + lane * ldt + 32 * blk;
  const float4* b4 = reinterpret_cast<const float4*>(e.bias + n);
  float4 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 x = *reinterpret_cast<const float4*>(src + 4 * q);
    const float4 b = e.bias ? b4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    v[q] = gelu_erf4(make_float4(x.x + b.x, x.y + b.y, x.z + b.z, x.w + b.w));
  }
  float amax = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[q].x), fabsf(v[q].y)), fmaxf(fabsf(v[q].z), fabsf(v[q].w))));
  const int ex = mx8_exp(amax);
  const float is = mx8_inv_scale(ex);
  uint32_t w[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) w[q] = mx8_pack4(v[q].x * is, v[q].y * is, v[q].z * is, v[q].w * is);
  if (m < M) {
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(e.out) + (long)m * e.ldc + n);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    e.out2[(long)m * e.ldc2 + (n >> 5)] = (uint8_t)(ex + 127);
  }
}

template <DT T, int KIND>
__device__ inline void epi_image64(const Epi& e, const float* img, int ldt, int mb, int n0, int M, int N, int tid,
                                   const float4* bpre = nullptr, const Resid8* pre = nullptr) {
  if constexpr (KIND == EPI_CROSSKV) {  // specialised cross-K/V launch (host: d % 256 == 0, xt % 4 == 0)
    if (((n0 / e.d) & 1) == 0) {
      epi_rows64<T, EPI_CROSSKV>(e, img, ldt, mb, n0, M, N, tid, bpre);
    } else {  // V^T: 4 consecutive keys of one column per 8-byte store
      const int col = tid & 255, r4 = (tid >> 8) * 4, n = n0 + col;
      const float b = e.bias ? e.bias[n] : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rr = r4 + 8 * u, m = mb + rr;
        if (m >= M) continue;
        u16x4 h;
#pragma unroll
        for (int q = 0; q < 4; ++q) h[q] = from_f32<T>(img[(rr + q) * ldt + col] + b);
        *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + crosskv_index(e, m, n)) = h;
      }
    }
    return;
  } else if constexpr (KIND == EPI_RESID32_LNS || KIND == EPI_GELU_POS32_LNS) {
    epi_rows64_lns<T, KIND>(e, img, ldt, mb, n0, M, tid, bpre, pre);
    return;
  } else if constexpr (KIND >= 0) {  // specialised launch: the host checked the vector conditions
    epi_rows64<T, KIND>(e, img, ldt, mb, n0, M, N, tid, bpre, pre);
    return;
  }
  const bool vec = (N & 3) == 0 && (e.ldc & 3) == 0;
  const bool kpart = e.kind == EPI_CROSSKV && ((n0 / e.d) & 1) == 0;  // K image: row-major 64-wide head rows
  if (vec || kpart) {
    switch (e.kind) {
      case EPI_STORE16: epi_rows64<T, EPI_STORE16>(e, img, ldt, mb, n0, M, N, tid); return;
      case EPI_GELU16: epi_rows64<T, EPI_GELU16>(e, img, ldt, mb, n0, M, N, tid); return;
      case EPI_RESID32: epi_rows64<T, EPI_RESID32>(e, img, ldt, mb, n0, M, N, tid); return;
      case EPI_GELU_POS32: epi_rows64<T, EPI_GELU_POS32>(e, img, ldt, mb, n0, M, N, tid); return;
      case EPI_STORE32: epi_rows64<T, EPI_STORE32>(e, img, ldt, mb, n0, M, N, tid); return;
      case EPI_GELU_MX8: epi_rows64<T, EPI_GELU_MX8>(e, img, ldt, mb, n0, M, N, tid); return;
      case EPI_CROSSKV:
        if (kpart) {
          epi_rows64<T, EPI_CROSSKV>(e, img, ldt, mb, n0, M, N, tid);
          return;
        }
        break;
      default: break;
    }
  }
  epi_from_image<T, 256, 512>(e, img, ldt, 64, mb, n0, M, N, tid);
}

// 64-row x 128-column image, 512 threads: a thread owns column quad (tid & 31) and rows (tid >> 5) + 16u
template <DT T, int KIND>
__device__ inline void epi_rows64_n128(const Epi& e, const float* img, int ldt, int mb, int n0, int M, int N, int tid,
                                      const float4* bpre = nullptr) {
  const int c4 = (tid & 31) * 4, r0 = tid >> 5;
  const int n = n0 + c4;
  if (n >= N) return;
  float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bpre)
    b = *bpre;
  else if (e.bias)
    b = *reinterpret_cast<const float4*>(e.bias + n);
  float4 v[4], aux[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = r0 + 16 * u, m = mb + row;
    v[u] = *reinterpret_cast<const float4*>(img + row * ldt + c4);
    v[u] = make_float4(v[u].x + b.x, v[u].y + b.y, v[u].z + b.z, v[u].w + b.w);
    if (KIND == EPI_RESID32 && m < M)
      aux[u] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(e.out) + (long)m * e.ldc + n);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int m = mb + r0 + 16 * u;
    if (m >= M) continue;  // uniform over each 32-lane half (same row)
    float4 x = v[u];
    if (KIND == EPI_GELU_MX8) {
      x = gelu_erf4(x);
      const int ex = mx8_exp(max8_lanes(fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)))));
      const float is = mx8_inv_scale(ex);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(e.out) + (long)m * e.ldc + n) =
          mx8_pack4(x.x * is, x.y * is, x.z * is, x.w * is);
      if ((tid & 7) == 0) e.out2[(long)m * e.ldc2 + (n >> 5)] = (uint8_t)(ex + 127);
    } else if (KIND == EPI_STORE16) {
      const u16x4 h = {from_f32<T>(x.x), from_f32<T>(x.y), from_f32<T>(x.z), from_f32<T>(x.w)};
      *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + (long)m * e.ldc + n) = h;
    } else {
      if (KIND == EPI_RESID32) x = make_float4(x.x + aux[u].x, x.y + aux[u].y, x.z + aux[u].z, x.w + aux[u].w);
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(e.out) + (long)m * e.ldc + n) = x;
    }
  }
}

template <DT T>
__device__ inline void epi_image64_n128(const Epi& e, const float* img, int ldt, int mb, int n0, int M, int N,
                                        int tid, const float4* bpre = nullptr) {
  switch (e.kind) {  // the host allows only these kinds, with N and ldc multiples of 4
    case EPI_STORE16: epi_rows64_n128<T, EPI_STORE16>(e, img, ldt, mb, n0, M, N, tid, bpre); break;
    case EPI_RESID32: epi_rows64_n128<T, EPI_RESID32>(e, img, ldt, mb, n0, M, N, tid, bpre); break;
    case EPI_STORE32: epi_rows64_n128<T, EPI_STORE32>(e, img, ldt, mb, n0, M, N, tid, bpre); break;
    case EPI_GELU_MX8: epi_rows64_n128<T, EPI_GELU_MX8>(e, img, ldt, mb, n0, M, N, tid, bpre); break;
    default: break;
  }
}

template <DT T, int KIND>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(const uint16_t* __restrict__ A, long lda,
                                                         const uint16_t* __restrict__ W, long ldw, int M, int N, int K,
                                                         Epi e) {
  constexpr int BM = 256, BN = 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesN = (N + BN - 1) / BN;
  const int tilesM = (M + BM - 1) / BM;
  const int nwg = tilesN * tilesM;
  // persistent: a workgroup walks tiles blockIdx.x, + gridDim.x, ... (gridDim.x a multiple of 8, so a tile stays on
  // the XCD the remap below assumes); the previous tile's epilogue stores drain while the next tile's first
  // slices are in flight, and the workgroup's LDS is not released and re-acquired per tile
  for (int tile = blockIdx.x; tile < nwg; tile += gridDim.x) {
  int bid = tile;
  {  // bijective XCD remap (§5.5 T1): each XCD gets a contiguous range of tiles
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  // grouped order inside that range: 4 row panels walk the columns together, so the ~32 tiles an XCD runs at
  // once share 4 A panels and ~8 W panels in its L2 (row-major order shared 2 A panels but 16+ W panels; 8 panels:
  // qkv alone 5 % faster, the encoder pass unchanged, profiles/r05t_g256_gm/)
  constexpr int GM = 4;
  const int gsz = GM * tilesN;
  const int grp = bid / gsz, gr = bid - grp * gsz;
  const int gm = min(GM, tilesM - grp * GM);
  const int tm = grp * GM + gr % gm, tn = gr / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  // this thread's epilogue column quad (n0 + 4 (tid & 63)) of the bias, loaded now so its latency hides behind
  // the main loop (the epilogue's column quads are the same in all four rounds)
  // (direct epilogue kinds: the lane's column quad after the in-quad transpose, wn 64 + 16 (fr & 3) + 4 (fr >> 2))
  // LayerNorm-folded consumers (encoder): out = rstd_m (acc - mean_m c1[n]) + c2[n] with c2 passed as the bias;
  // (mean, rstd) of the tile's 256 rows are merged from the producer's per-256-column statistics at tile start
  // into LDS past the ring, and c1's column quad is loaded with the bias
  constexpr bool kLnf = KIND == EPI_LNF_STORE16 || KIND == EPI_LNF_GELU16;
  constexpr bool kGelu = KIND == EPI_GELU16 || KIND == EPI_LNF_GELU16;
  constexpr bool kDirect = kLnf || KIND == EPI_STORE16 || KIND == EPI_GELU16;
  const int bcol = kDirect ? (wave & 3) * 64 + 16 * (lane & 3) + 4 * ((lane >> 2) & 3) : 4 * (tid & 63);
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f), c14 = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (kLnf) {
    // the tile's raw statistics go to LDS by DMA ahead of the ring's first slices (wave g < lng: group g's 256 rows,
    // two 1 KiB pieces; rows past M clamped, never stored), so the counted vmcnt of the main loop covers them and no
    // VGPR load is waited for; merged after the loop
    if (wave < e.lng) {
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        const int mr = min(m0 + 128 * pc + 2 * lane, M - 2);
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(e.stats + (long)wave * e.stats_ld + mr),
            (__attribute__((address_space(3))) void*)(smem + kG256StatRaw + (wave * 256 + 128 * pc) * 8), 16, 0, 0);
      }
    }
    const int bc = min(n0 + bcol, N - 4);
    bias4 = *reinterpret_cast<const float4*>(e.bias + bc);
    c14 = *reinterpret_cast<const float4*>(e.c1 + bc);
  } else if (KIND >= 0 && e.bias && n0 + bcol < N) {
    bias4 = *reinterpret_cast<const float4*>(e.bias + n0 + bcol);
  }

  // Half-tile ring (the geometry of cdna_hip_programming.md §5's 256² template): K-tiles of 64 (128-B rows = whole
  // cache lines, where the 32-deep slices below fetch every line in two halves one slice apart) in two 64 KiB buffers
  // (t & 1) of four 16 KiB units, each 128 rows x 128 B:
  //   unit 0 = A rows m0 + 128 wm + [0, 64)   (quadrant row 0 of every wave)    read in phase 0
  //   unit 1 = W rows n0 + 64 wn + [0, 32)    (quadrant column 0)                read in phases 0 and 3
  //   unit 2 = W rows n0 + 64 wn + [32, 64)   (quadrant column 1)                read in phase 1
  //   unit 3 = A rows m0 + 128 wm + [64, 128) (quadrant row 1)                   read in phase 2
  // Phase p of K-tile t: [LDS reads of its unit(s) + 2 DMAs of one unit] s_barrier [16 MFMAs: one 64 x 32 quadrant
  // of the wave's 128 x 64 tile, K = 64] s_barrier, quadrants (0,0) (0,1) (1,1) (1,0); waves 4..7 one barrier behind.
  // A unit is restaged one phase after its last read (every memory segment retires its reads before its barrier):
  // phase 0 stages unit 1 of K-tile t + 1, phases 1..3 units 0, 2, 3 of K-tile t + 2; one counted wait per K-tile,
  // vmcnt(6) in phase 3 (the three units of t + 2 may fly), completes K-tile t + 1 three to six phases after issue.
  // Row r of a unit sits at r * 128 B with its 16-B chunk c at position c ^ ((r >> 1) & 7): a fragment read (16 rows
  // fr, chunk 4s + fq) puts every ds_read_b128 lane group on 16 distinct (r & 1, position) pairs = all 64 banks.
  const int nk = K >> 6;
  uint32_t uoff[4][2];  // element offsets from A (units 0, 3) or W (units 1, 2) of this lane's two pieces (w, w + 8)
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = 8 * (wave + 8 * j) + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (u == 0 || u == 3) {
        const int m = min(m0 + (r >> 6) * 128 + (u == 3 ? 64 : 0) + (r & 63), M - 1);
        uoff[u][j] = (uint32_t)((long)m * lda + c * 8);
      } else {
        const int n = min(n0 + (r >> 5) * 64 + (u == 2 ? 32 : 0) + (r & 31), N - 1);
        uoff[u][j] = (uint32_t)((long)n * ldw + c * 8);
      }
    }
  auto issue_unit = [&](int t, int u) {
    char* dst = smem + (t & 1) * 65536 + u * 16384;
    const uint16_t* base = (u == 0 || u == 3) ? A : W;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + uoff[u][j] + (long)t * 64),
                                       (__attribute__((address_space(3))) void*)(dst + (wave + 8 * j) * 1024), 16, 0,
                                       0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  const int fr = lane & 15, fq = lane >> 4;
  const int sw0 = (fq ^ (fr >> 1)) << 4, sw1 = ((4 + fq) ^ (fr >> 1)) << 4;
  const int arow = (wm * 64 + fr) * 128, brow = (wn * 32 + fr) * 128;
  u16x8 af[4][2], bfr[2][2];
  auto read_a = [&](const char* U) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      af[ii][0] = *reinterpret_cast<const u16x8*>(U + arow + ii * 2048 + sw0);
      af[ii][1] = *reinterpret_cast<const u16x8*>(U + arow + ii * 2048 + sw1);
    }
  };
  auto read_b = [&](const char* U) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      bfr[jj][0] = *reinterpret_cast<const u16x8*>(U + brow + jj * 2048 + sw0);
      bfr[jj][1] = *reinterpret_cast<const u16x8*>(U + brow + jj * 2048 + sw1);
    }
  };
  auto quadrant = [&](int g, int h) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[4 * g + ii][2 * h + jj] = WMX_G256_MFMA(af[ii][s], bfr[jj][s], acc[4 * g + ii][2 * h + jj]);
  };
  // prologue: K-tile 0 whole, then units 0, 2, 3 of K-tile 1 (its unit 1 goes out in phase 0 of K-tile 0)
#pragma unroll
  for (int u = 0; u < 4; ++u) issue_unit(0, u);
  if (nk > 1) {
    issue_unit(1, 0);
    issue_unit(1, 2);
    issue_unit(1, 3);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  const bool lagging = __builtin_amdgcn_readfirstlane(wave) >= 4;
  if (lagging) __builtin_amdgcn_s_barrier();
  // static priority 1 for the lagging half (MI355X_MICROARCH.md "two waves per SIMD" item 4; s_setprio around every
  // segment measured 1.0-1.4 % slower per encoder pass, profiles/r03zs_static_prio/)
  if (lagging) __builtin_amdgcn_s_setprio(1);
#define WMX_G256_SEG(QG, QH)                                 \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");         \
  __builtin_amdgcn_sched_barrier(0);                         \
  __builtin_amdgcn_s_barrier();                              \
  WMX_G256_PIN;                                              \
  quadrant(QG, QH);                                          \
  __builtin_amdgcn_sched_barrier(0);                         \
  __builtin_amdgcn_s_barrier();
  for (int t = 0; t < nk; ++t) {
    const char* U = smem + (t & 1) * 65536;
    read_a(U);  // phase 0: units 0 and 1
    read_b(U + 16384);
    if (t + 1 < nk) issue_unit(t + 1, 1);
    WMX_G256_SEG(0, 0)
    read_b(U + 2 * 16384);  // phase 1: unit 2
    if (t + 2 < nk) issue_unit(t + 2, 0);
    WMX_G256_SEG(0, 1)
    read_a(U + 3 * 16384);  // phase 2: unit 3
    if (t + 2 < nk) issue_unit(t + 2, 2);
    WMX_G256_SEG(1, 1)
    read_b(U + 16384);  // phase 3: unit 1 again
    if (t + 2 < nk) {
      issue_unit(t + 2, 3);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // K-tile t + 1 complete
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    WMX_G256_SEG(1, 0)
  }
#undef WMX_G256_SEG
  if (!lagging) __builtin_amdgcn_s_barrier();
  __syncthreads();
  if constexpr (kLnf) {  // Chan merge of the equal-count (256-column) groups of each of the tile's rows
    if (tid < 256) {
      const float2* raw = reinterpret_cast<const float2*>(smem + kG256StatRaw);
      float mean = 0.f;
      for (int g = 0; g < e.lng; ++g) mean += raw[g * 256 + tid].x;
      mean /= (float)e.lng;
      float m2 = 0.f;
      for (int g = 0; g < e.lng; ++g) {
        const float2 v = raw[g * 256 + tid];
        const float dm = v.x - mean;
        m2 += v.y + 256.f * dm * dm;
      }
      reinterpret_cast<float2*>(smem + kG256StatRow)[tid] =
          make_float2(mean, 1.0f / sqrtf(m2 / (256.f * (float)e.lng) + 1e-5f));
    }
    __syncthreads();
  }
  if constexpr (kDirect) {
    // LDS-free epilogue: for every (fragment row i, register r) the 16 lanes of a row group hold columns
    // 16 j + fr (j = 0..3) of one output row; a 4 x 4 transpose inside each lane quad (lane-dependent register
    // rotation, three DPP quad rotations, rotation back) leaves lane (fr) with the 4 consecutive columns
    // wn 64 + 16 (fr & 3) + 4 (fr >> 2) .. +3, stored as one 8-byte bf16 quad.  No image, no barriers.
    const int q = lane & 3;
    const int n = n0 + bcol;
    {  // every lane takes part in the DPP exchanges; only the stores are guarded
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float4 lsr[2];
        if constexpr (kLnf) {
          const float4* l4 = reinterpret_cast<const float4*>(smem + kG256StatRow) + (wm * 128 + i * 16 + fq * 4) / 2;
          lsr[0] = l4[0];
          lsr[1] = l4[1];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 128 + i * 16 + fq * 4 + r;
          float v0 = acc[i][0][r], v1 = acc[i][1][r], v2 = acc[i][2][r], v3 = acc[i][3][r];
          // u[k] = v[(q + k) & 3]
          if (q & 1) {
            const float t = v0;
            v0 = v1, v1 = v2, v2 = v3, v3 = t;
          }
          if (q & 2) {
            float t = v0;
            v0 = v2, v2 = t;
            t = v1, v1 = v3, v3 = t;
          }
          // u'[k] = u[k] of quad lane (q - k) & 3
          v1 = dpp_mov<0x93>(v1);  // quad_perm [3,0,1,2]
          v2 = dpp_mov<0x4E>(v2);  // quad_perm [2,3,0,1]
          v3 = dpp_mov<0x39>(v3);  // quad_perm [1,2,3,0]
          // w[m] = u'[(q - m) & 3] = x[(m - q) & 3] with x = (u'0, u'3, u'2, u'1)
          float x0 = v0, x1 = v3, x2 = v2, x3 = v1;
          if (q & 1) {
            const float t = x3;
            x3 = x2, x2 = x1, x1 = x0, x0 = t;
          }
          if (q & 2) {
            float t = x0;
            x0 = x2, x2 = t;
            t = x1, x1 = x3, x3 = t;
          }
          float4 o;
          if constexpr (kLnf) {
            const float2 ls = (r & 1) ? make_float2(lsr[r >> 1].z, lsr[r >> 1].w) : make_float2(lsr[r >> 1].x, lsr[r >> 1].y);
            o = make_float4(ls.y * (x0 - ls.x * c14.x) + bias4.x, ls.y * (x1 - ls.x * c14.y) + bias4.y,
                            ls.y * (x2 - ls.x * c14.z) + bias4.z, ls.y * (x3 - ls.x * c14.w) + bias4.w);
          } else {
            o = make_float4(x0 + bias4.x, x1 + bias4.y, x2 + bias4.z, x3 + bias4.w);
          }
          if (kGelu) o = gelu_erf4(o);  // packed: the epilogue runs outside the MFMA shadow
          if (m < M && n < N) {
            const u16x4 h = {from_f32<T>(o.x), from_f32<T>(o.y), from_f32<T>(o.z), from_f32<T>(o.w)};
            *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + (long)m * e.ldc + n) = h;
          }
        }
      }
    }
    __syncthreads();  // the next tile's DMA must not overwrite the ring before every wave left this tile
    continue;
  }
  // epilogue: 4 rounds of 64 rows through an fp32 LDS image [64][BN + 4]; the residual-RMW kinds load the next
  // round's residual rows while this round runs
  constexpr int LDT = BN + 4;
  constexpr bool kPre = KIND == EPI_RESID32 || KIND == EPI_RESID32_LNS;
  float* img = reinterpret_cast<float*>(smem);
  Resid8 pre;  // one buffer: round rd + 1's rows are requested as soon as round rd has consumed its own (double
              // buffering spilled: the prologue's reloads drained the DMA pipeline with vmcnt(0))
  if constexpr (kPre) resid_load<KIND>(pre, e, m0, n0, M, tid);
#pragma unroll
  for (int rd = 0; rd < 4; ++rd) {
    if (wm == (rd >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = (rd & 1) * 4 + ii;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) img[(ii * 16 + fq * 4 + r) * LDT + wn * 64 + j * 16 + fr] = acc[i][j][r];
        }
      }
    }
    __syncthreads();
    epi_image64<T, KIND>(e, img, LDT, m0 + rd * 64, n0, M, N, tid, &bias4, kPre ? &pre : nullptr);
    if constexpr (kPre) {
      if (rd < 3) resid_load<KIND>(pre, e, m0 + (rd + 1) * 64, n0, M, tid);
    }
    __syncthreads();
  }
  }  // tile loop
}

// ------------------------------------------------------------------------------------------------
// MX-fp8 GEMM: 256 (M) x 128 (N) tile, 8 waves (4 M x 2 N, wave tile 64 x 64 = 4 x 4 fragments: 64 accumulator
// + 64 operand VGPRs, no spills at two waves per SIMD), K staged in 128-deep slices (128 B of e4m3 per row)
// through a 3-slot LDS ring by global_load_lds (16-B chunk c of row r at c ^ (r & 7)); the slice's e8m0 scales
// are one dword per row (its four 32-blocks).  v_mfma_scale_f32_16x16x128_f8f6f4 takes lane l = (r = l & 15,
// g = l >> 4) as row r with k = 16g .. +15 and 64 + 16g .. +15 (chunks g and g + 4 of the row), and its scale
// operand as the scale of block g of row r (tools/mx8_check.hip measures both maps).
// Ping-pong phase schedule as gemm256_kernel; slice t + 2 is in flight while slice t computes: each wave issues
// 7 DMAs per slice (4 A pieces + the scale dword in phase A, 2 W pieces in phase B) and waits for slice t + 1 with
// a counted vmcnt(7) right before the barrier that precedes the first read of it by either wave half.
// ------------------------------------------------------------------------------------------------
constexpr int kMx8ARows = 256 * 128, kMx8WRows = 128 * 128;
constexpr int kMx8Slot = kMx8ARows + kMx8WRows + 512 * 4;  // + scale dwords: 256 A rows, 128 W rows, 128 spare
constexpr int kMx8Lds = 3 * kMx8Slot;                       // 150 KiB

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <DT T>
__global__ __launch_bounds__(512, 1) void gemm_mx8_kernel(const uint8_t* __restrict__ A, long lda,
                                                          const uint8_t* __restrict__ AS, long ldas,
                                                          const uint8_t* __restrict__ W, long ldw,
                                                          const uint8_t* __restrict__ WS, long ldws, int M, int N,
                                                          int K, Epi e) {
  constexpr int BM = 256, BN = 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesN = (N + BN - 1) / BN;
  const int tilesM = (M + BM - 1) / BM;
  const int nwg = tilesN * tilesM;
  // persistent over tiles, as gemm256_kernel (gridDim.x a multiple of 8)
  for (int tile = blockIdx.x; tile < nwg; tile += gridDim.x) {
  int bid = tile;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GM = 4;
  const int gsz = GM * tilesN;
  const int grp = bid / gsz, gr = bid - grp * gsz;
  const int gm = min(GM, tilesM - grp * GM);
  const int tm = grp * GM + gr % gm, tn = gr / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  // the epilogue's bias column quad (n0 + 4 (tid & 31)), loaded at tile start
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e.bias && n0 + 4 * (threadIdx.x & 31) < N) bias4 = *reinterpret_cast<const float4*>(e.bias + n0 + 4 * (threadIdx.x & 31));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nk = K >> 7;

  // staging (8-row x 128-B pieces): wave w issues A pieces w + 8j (j < 4) and W pieces w + 8j (j < 2); scale
  // dwords: wave w stages rows 64w .. 64w + 63 of [256 A rows | 128 W rows | 128 spare] (waves 6, 7 re-read W
  // rows into the spare area so that every wave issues the same 7 DMAs per slice)
  const int srow = lane >> 3;
  const int scol = ((lane & 7) ^ srow) * 16;
  int aoff[4], woff[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) aoff[j] = (int)min((long)min(m0 + (wave + 8 * j) * 8 + srow, M - 1) * lda, 0x7fffffffL);
#pragma unroll
  for (int j = 0; j < 2; ++j) woff[j] = (int)((long)min(n0 + (wave + 8 * j) * 8 + srow, N - 1) * ldw);
  const uint8_t* ssrc = wave < 4 ? AS + (long)min(m0 + 64 * wave + lane, M - 1) * ldas
                                 : WS + (long)min(n0 + 64 * ((wave - 4) & 1) + lane, N - 1) * ldws;
  const int sdst = kMx8ARows + kMx8WRows + wave * 256;
  auto issue_a = [&](int kt) {
    char* slot = smem + (kt % 3) * kMx8Slot;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(A + aoff[j] + scol + kt * 128),
                                       (__attribute__((address_space(3))) void*)(slot + (wave + 8 * j) * 1024), 16, 0,
                                       0);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ssrc + kt * 4),
                                     (__attribute__((address_space(3))) void*)(slot + sdst), 4, 0, 0);
  };
  auto issue_w = [&](int kt) {
    char* slot = smem + (kt % 3) * kMx8Slot;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(W + woff[j] + scol + kt * 128),
                                       (__attribute__((address_space(3))) void*)(slot + kMx8ARows +
                                                                                 (wave + 8 * j) * 1024),
                                       16, 0, 0);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  const int fr = lane & 15, g = lane >> 4;
  const int c0 = (g ^ (fr & 7)) << 4, c1 = ((g + 4) ^ (fr & 7)) << 4;
  const int arow = wm * 64 + fr, brow = wn * 64 + fr;
  auto frag = [&](const char* base, int row) {
    const i32x4 lo = *reinterpret_cast<const i32x4*>(base + row * 128 + c0);
    const i32x4 hi = *reinterpret_cast<const i32x4*>(base + row * 128 + c1);
    return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

  issue_a(0);
  issue_w(0);
  if (nk > 1) {
    issue_a(1);
    issue_w(1);
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  const bool lagging = __builtin_amdgcn_readfirstlane(wave) >= 4;
  if (lagging) __builtin_amdgcn_s_barrier();
  if (lagging) __builtin_amdgcn_s_setprio(1);  // static priority for the lagging half (as gemm256)
  i32x8 af[2], bfr[4];
  int sa[2], sb[4];
  for (int t = 0; t < nk; ++t) {
    const char* S = smem + (t % 3) * kMx8Slot;
    const char* Wb = S + kMx8ARows;
    const uint32_t* SA = reinterpret_cast<const uint32_t*>(S + kMx8ARows + kMx8WRows);
    const uint32_t* SB = SA + 256;
    const bool more = t + 2 < nk;
    // ---- phase A: B fragments 0..3, A fragments 0, 1; A half (+ scales) of slice t + 2 ----
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bfr[j] = frag(Wb, brow + 16 * j);
      sb[j] = (int)(SB[brow + 16 * j] >> (8 * g));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[i] = frag(S, arow + 16 * i);
      sa[i] = (int)(SA[arow + 16 * i] >> (8 * g));
    }
    if (more) issue_a(t + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, sa[i], 0,
                                                                     sb[j]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase B: A fragments 2, 3; W half of slice t + 2 ----
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[i] = frag(S, arow + 16 * (i + 2));
      sa[i] = (int)(SA[arow + 16 * (i + 2)] >> (8 * g));
    }
    if (more) issue_w(t + 2);
    if (lagging) {  // slice t + 1 complete before the barrier ahead of its first read (slice t + 2 may fly)
      if (more)
        asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i + 2][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i + 2][j], 0, 0, 0, sa[i],
                                                                         0, sb[j]);
    if (!lagging) {  // the same barrier, seen from the leading half
      if (more)
        asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  if (!lagging) __builtin_amdgcn_s_barrier();
  __syncthreads();

  // epilogue: 4 rounds of 64 rows (one wave row each) through an fp32 LDS image [64][BN + 4]
  constexpr int LDT = BN + 4;
  float* img = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int rd = 0; rd < 4; ++rd) {
    if (wm == rd) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) img[(i * 16 + g * 4 + r) * LDT + wn * 64 + j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    epi_image64_n128<T>(e, img, LDT, m0 + rd * 64, n0, M, N, tid, &bias4);
    __syncthreads();
  }
  }  // tile loop
}

// ------------------------------------------------------------------------------------------------
// MX-fp8 GEMM, 256 x 256 tile (the gemm256 structure at the fp8 rate): v_mfma_scale_f32_32x32x64_f8f6f4 takes K = 64
// per instruction, so a 64-deep slice is 64 bytes of e4m3 per row -- the same 32 KiB slot, 1 KiB pieces and
// source-side swizzle as the bf16 ring -- plus the slice's two e8m0 scale bytes per row (A then W, 1 KiB, staged
// by one dword-per-lane DMA per wave: the dword holding this slice's two bytes).  8 waves (2 M x 4 N), wave tile 128 x 64 = 4 x 2 blocks of 32 x 32 (f32x16
// accumulators), two phases per slice of 4 MFMAs (64 cycles each) with the ping-pong stagger of gemm256, 4 slots.
// Fragment of 32 rows: lane l holds row (l & 31), k = 16g .. 16g + 15 in bytes 0..15 and 32 + 16g .. in bytes
// 16..31 (g = l >> 5), i.e. 16-B pieces g and 2 + g of its 64-B row; its scale operand is the byte of (row l & 31,
// 32-k block g) (tools/mx8_check32.hip measures both maps).  Epilogues through the 64 x 256 fp32 LDS image.
// ------------------------------------------------------------------------------------------------
constexpr int kMx8bLds = 4 * 32768 + 2 * 2048;  // 132 KiB: two 64 KiB unit buffers + two 2 KiB scale buffers
static_assert(kMx8bLds <= 163840 && 64 * (256 + 4) * 4 <= kMx8bLds, "gemm_mx8_256 LDS");

template <DT T, int KIND>
__global__ __launch_bounds__(512, 1) void gemm_mx8_256_kernel(const uint8_t* __restrict__ A, long lda,
                                                              const uint8_t* __restrict__ AS, long ldas,
                                                              const uint8_t* __restrict__ W, long ldw,
                                                              const uint8_t* __restrict__ WS, long ldws, int M, int N,
                                                              int K, Epi e) {
  constexpr int BM = 256, BN = 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesN = (N + BN - 1) / BN;
  const int tilesM = (M + BM - 1) / BM;
  const int nwg = tilesN * tilesM;
  for (int tile = blockIdx.x; tile < nwg; tile += gridDim.x) {
  int bid = tile;
  {  // bijective XCD remap, then 4 row panels walk the columns together (as gemm256)
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GM = 4;
  const int gsz = GM * tilesN;
  const int grp = bid / gsz, gr = bid - grp * gsz;
  const int gm = min(GM, tilesM - grp * GM);
  const int tm = grp * GM + gr % gm, tn = gr / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);  // (loaded after the main loop: no VGPRs to spare inside)

  // 128-deep half-tile ring (as gemm256's 64-deep one): a K-tile is 128 e4m3 = one 128-B line per row,
  // four 16 KiB units of 128 rows in two buffers (unit 0 = A rows m0 + 128 wm + [0, 64), 1 = W rows n0 + 64 wn +
  // [0, 32), 2 = W rows n0 + 64 wn + [32, 64), 3 = A rows m0 + 128 wm + [64, 128)) plus the K-tile's scale dword of
  // every row (4 e8m0 bytes) in a 2 KiB buffer per K-tile, staged with unit 1.  Phase p: one 64 x 32 quadrant of the
  // wave's 128 x 64 tile (2 A blocks x 1 W block x 2 K-steps = 4 MFMAs of 64 cycles), quadrants (0,0) (0,1) (1,1)
  // (1,0); unit 1 + scales of K-tile t + 1 in phase 0, units 0, 2, 3 of t + 2 in phases 1..3, one vmcnt(6) per
  // K-tile.  Row r holds chunk c at c ^ ((r >> 1) & 7): conflict-free for the 32-row fragments' lane groups.
  const int nk = K >> 7;
  // this lane's unit row (pieces w and w + 8) and swizzled source chunk; the row offsets are recomputed per issue
  // (the f32x16 accumulators leave no room for eight resident offsets)
  const int ur = 8 * wave + (lane >> 3);
  const int uc = ((lane & 7) ^ ((ur >> 1) & 7)) * 16;  // (ur + 64) has the same (r >> 1) & 7
  // unit rows: A (units 0, 3) m0 + ur + 128 j + 64 [u == 3]; W (units 1, 2) n0 + 64 (ur >> 5) + (ur & 31) + 128 j +
  // 32 [u == 2] (N % 256 == 0 here: W rows need no clamp)
  const int arb = m0 + ur, wrb = n0 + 64 * (ur >> 5) + (ur & 31);
  // scales: wave w < 4 stages A rows 64 w + lane, wave w >= 4 W rows 64 (w - 4) + lane (K-tile t: dword t of the row)
  const uint8_t* ssrc = wave < 4 ? AS + (long)min(m0 + 64 * wave + lane, M - 1) * ldas
                                 : WS + (long)min(n0 + 64 * (wave - 4) + lane, N - 1) * ldws;
  constexpr int kSc = 4 * 32768;  // scale buffers after the two 64 KiB unit buffers
  auto issue_unit = [&](int t, int u) {
    char* dst = smem + (t & 1) * 65536 + u * 16384;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      // the row base goes through an empty asm per issue, so the compiler recomputes the row instead of holding
      // eight row pointers across the K loop (they spilled beside the f32x16 accumulators)
      int rb = (u == 0 || u == 3) ? arb : wrb;
      asm volatile("" : "+v"(rb));
      const uint8_t* src;
      if (u == 0 || u == 3)
        src = A + (long)min(rb + 128 * j + (u == 3 ? 64 : 0), M - 1) * lda;
      else
        src = W + (long)(rb + 128 * j + (u == 2 ? 32 : 0)) * ldw;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + uc + (long)t * 128),
                                       (__attribute__((address_space(3))) void*)(dst + (wave + 8 * j) * 1024), 16, 0,
                                       0);
    }
  };
  auto issue_scales = [&](int t) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ssrc + (long)t * 4),
                                     (__attribute__((address_space(3))) void*)(smem + kSc + (t & 1) * 2048 + wave * 256),
                                     4, 0, 0);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int fr = lane & 31, g = lane >> 5;
  const int sw = (fr >> 1) & 7;
  // K-step s of a fragment: 16-B chunks 4 s + g and 4 s + 2 + g of the lane's row (bytes 16 g.. and 32 + 16 g..)
  // chunk 4 s + 2 h + g sits at ((4 s + 2 h + g) ^ sw) << 4 = (((g ^ sw) << 4) ^ (64 s + 32 h)): the row base plus
  // the step-0 chunk offset, XORed (row bases are multiples of 128)
  const int q00 = (g ^ sw) << 4;
  const int arow = (wm * 64 + fr) * 128, brow = (wn * 32 + fr) * 128;
  const int sarow = (wm * 128 + fr) * 4 + g, sbrow = 1024 + (wn * 64 + fr) * 4 + g;
  i32x8 af[2][2], bfr[2];
  int sa[2][2], sb[2];
  auto frag2 = [&](const char* U, int off, i32x8& f0, i32x8& f1) {
    int o = off + q00;
    asm volatile("" : "+v"(o));
    const i32x4 a0 = *reinterpret_cast<const i32x4*>(U + o);
    const i32x4 a1 = *reinterpret_cast<const i32x4*>(U + (o ^ 32));
    const i32x4 b0 = *reinterpret_cast<const i32x4*>(U + (o ^ 64));
    const i32x4 b1 = *reinterpret_cast<const i32x4*>(U + (o ^ 96));
    f0 = i32x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    f1 = i32x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  };
  // A blocks 2 g2 + ii (ii = 0, 1) of unit 0 (g2 = 0) or 3 (g2 = 1), with their scale bytes (block 2 s + g of the tile)
  auto read_a = [&](const char* U, const char* SC, int g2) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      frag2(U, arow + ii * 4096, af[ii][0], af[ii][1]);
      const char* sp = SC + sarow + (64 * g2 + 32 * ii) * 4;
      sa[ii][0] = (int)*reinterpret_cast<const uint8_t*>(sp);
      sa[ii][1] = (int)*reinterpret_cast<const uint8_t*>(sp + 2);
    }
  };
  auto read_b = [&](const char* U, const char* SC, int h) {
    frag2(U, brow, bfr[0], bfr[1]);
    const char* sp = SC + sbrow + 32 * h * 4;
    sb[0] = (int)*reinterpret_cast<const uint8_t*>(sp);
    sb[1] = (int)*reinterpret_cast<const uint8_t*>(sp + 2);
  };
  auto quadrant = [&](int g2, int h) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
        acc[2 * g2 + ii][h] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[ii][s], bfr[s], acc[2 * g2 + ii][h], 0,
                                                                              0, 0, sa[ii][s], 0, sb[s]);
  };
  issue_scales(0);
#pragma unroll
  for (int u = 0; u < 4; ++u) issue_unit(0, u);
  if (nk > 1) {
    issue_unit(1, 0);
    issue_unit(1, 2);
    issue_unit(1, 3);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  const bool lagging = __builtin_amdgcn_readfirstlane(wave) >= 4;
  if (lagging) __builtin_amdgcn_s_barrier();
  if (lagging) __builtin_amdgcn_s_setprio(1);
#define WMX_MX8_SEG(QG, QH)                          \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
  __builtin_amdgcn_sched_barrier(0);                 \
  __builtin_amdgcn_s_barrier();                      \
  WMX_G256_PIN;                                      \
  quadrant(QG, QH);                                  \
  __builtin_amdgcn_sched_barrier(0);                 \
  __builtin_amdgcn_s_barrier();
  // one K-tile; I1 / I2: K-tile t + 1 / t + 2 exists.  The three forms are separate straight-line bodies: a
  // conditional issue inside the body let the compiler sink three phases' MFMAs past their barriers into the block
  // after the last branch (and spill the accumulators that then overlapped)
  auto ktile = [&](int t, auto I1, auto I2) {
    const char* U = smem + (t & 1) * 65536;
    const char* SC = smem + kSc + (t & 1) * 2048;
    read_a(U, SC, 0);  // phase 0: units 0 and 1
    read_b(U + 16384, SC, 0);
    if constexpr (decltype(I1)::value) {
      issue_unit(t + 1, 1);
      issue_scales(t + 1);
    }
    WMX_MX8_SEG(0, 0)
    read_b(U + 2 * 16384, SC, 1);  // phase 1: unit 2
    if constexpr (decltype(I2)::value) issue_unit(t + 2, 0);
    WMX_MX8_SEG(0, 1)
    read_a(U + 3 * 16384, SC, 1);  // phase 2: unit 3
    if constexpr (decltype(I2)::value) issue_unit(t + 2, 2);
    WMX_MX8_SEG(1, 1)
    read_b(U + 16384, SC, 0);  // phase 3: unit 1 again
    if constexpr (decltype(I2)::value) {
      issue_unit(t + 2, 3);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // K-tile t + 1 complete (unit 1 + scales, then 0, 2, 3)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    WMX_MX8_SEG(1, 0)
  };
  using Yes = std::integral_constant<bool, true>;
  using No = std::integral_constant<bool, false>;
  for (int t = 0; t + 2 < nk; ++t) ktile(t, Yes{}, Yes{});
  if (nk >= 2) ktile(nk - 2, Yes{}, No{});
  ktile(nk - 1, No{}, No{});
  // anchor every accumulator here: the epilogue reads each one inside a wave-row branch, where the compiler would
  // otherwise sink the last K-tile's MFMAs (out of their barrier segments)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[i][j]));
#undef WMX_MX8_SEG
  if (e.bias && n0 + 4 * (tid & 63) < N) bias4 = *reinterpret_cast<const float4*>(e.bias + n0 + 4 * (tid & 63));
  if (!lagging) __builtin_amdgcn_s_barrier();
  __syncthreads();

  // epilogue: 4 rounds of 64 rows through the fp32 LDS image [64][BN + 4]; 32 x 32 block (i, j) register r of lane l
  // is row 32 i + 8 (r / 4) + 4 (l / 32) + r % 4, column 32 j + l % 32 of the wave tile
  constexpr int LDT = BN + 4;
  constexpr bool kPre = false;  // (the residual prefetch spilled here: 256 VGPRs with the f32x16 accumulators)
  float* img = reinterpret_cast<float*>(smem);
  Resid8 pre;
  if constexpr (kPre) resid_load<KIND>(pre, e, m0, n0, M, tid);
#pragma unroll
  for (int rd = 0; rd < 4; ++rd) {
    if (wm == (rd >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = (rd & 1) * 2 + ii;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            img[(ii * 32 + 8 * (r >> 2) + 4 * g + (r & 3)) * LDT + wn * 64 + j * 32 + fr] = acc[i][j][r];
      }
    }
    __syncthreads();
    if constexpr (KIND == EPI_GELU_MX8)
      epi_gelu_mx8_blocks<T>(e, img, LDT, m0 + rd * 64, n0, M, tid);
    else if constexpr (KIND == EPI_RESID32)  // (8 rows at once spilled beside the accumulators)
      epi_rows64<T, EPI_RESID32, 4>(e, img, LDT, m0 + rd * 64, n0, M, N, tid, &bias4);
    else
      epi_image64<T, KIND>(e, img, LDT, m0 + rd * 64, n0, M, N, tid, &bias4, kPre ? &pre : nullptr);
    if constexpr (kPre) {
      if (rd < 3) resid_load<KIND>(pre, e, m0 + (rd + 1) * 64, n0, M, tid);
    }
    __syncthreads();
  }
  }  // tile loop
}

static int g256_grid(int tiles);

// the 256 x 256 / 32x32x64 form for the encoder shapes (the 256 x 128 / 16x16x128 form for the others)
static bool mx8_256_ok(const Mx8Call& g) {
  return g.M >= 4096 && g.N % 256 == 0 && g.K % 64 == 0 && g.ldas % 2 == 0 && g.ldws % 2 == 0 &&
         (g.epi.kind == EPI_STORE16 || g.epi.kind == EPI_RESID32 || g.epi.kind == EPI_GELU_MX8);
}

template <DT T>
static void launch_mx8_t(const Mx8Call& g, hipStream_t st) {
  if (mx8_256_ok(g)) {
    const int tiles = g256_grid(((g.M + 255) / 256) * (g.N / 256));
#define WMX_MX8B_LAUNCH(KD)                                                                                         \
  hipLaunchKernelGGL((gemm_mx8_256_kernel<T, KD>), dim3(tiles), dim3(512), kMx8bLds, st, g.A, g.lda, g.AS, g.ldas, \
                     g.W, g.ldw, g.WS, g.ldws, g.M, g.N, g.K, g.epi)
    switch (g.epi.kind) {
      case EPI_STORE16: WMX_MX8B_LAUNCH(EPI_STORE16); break;
      case EPI_RESID32: WMX_MX8B_LAUNCH(EPI_RESID32); break;
      default: WMX_MX8B_LAUNCH(EPI_GELU_MX8); break;
    }
#undef WMX_MX8B_LAUNCH
    return;
  }
  const int tiles = ((g.M + 255) / 256) * ((g.N + 127) / 128);
  hipLaunchKernelGGL((gemm_mx8_kernel<T>), dim3(g256_grid(tiles)), dim3(512), kMx8Lds, st, g.A, g.lda, g.AS, g.ldas,
                     g.W, g.ldw, g.WS, g.ldws, g.M, g.N, g.K, g.epi);
}

void launch_gemm_mx8(DT dt, const Mx8Call& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return;
  WMX_CHECK(g.K % 128 == 0 && g.lda % 16 == 0 && g.ldw % 16 == 0 && g.ldas % 4 == 0 && g.ldws % 4 == 0,
            "gemm_mx8: K must be a multiple of 128, rows 16-B aligned");
  WMX_CHECK((g.epi.kind == EPI_STORE16 || g.epi.kind == EPI_RESID32 || g.epi.kind == EPI_STORE32 ||
             g.epi.kind == EPI_GELU_MX8) && g.N % 32 == 0 && g.epi.ldc % 4 == 0,
            "gemm_mx8: epilogue");
  if (dt == DT::BF16)
    launch_mx8_t<DT::BF16>(g, st);
  else
    launch_mx8_t<DT::F16>(g, st);
  WMX_HIP(hipGetLastError());
}

template <DT T>
__global__ __launch_bounds__(256) void gemm_splitk_reduce(const float* __restrict__ ws, int splits, int M, int N,
                                                          Epi e) {
  const long total = (long)M * N;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += ws[s * total + i];
    epi_store<T>(e, (int)(i / N), (int)(i % N), v);
  }
}

// ------------------------------------------------------------------------------------------------
// skinny GEMM for decode steps (M <= 256 rows = streams x beams): one workgroup = all M rows x 16 output
// columns; the 4 waves split K and their partial tiles are summed in LDS (deterministic, no split-K launch).
// Weights (the only large operand) stream once with 16-B loads, KU k-steps in flight per wave; activations are
// L2-resident and read as MFMA fragments directly.  N/16 workgroups (80-320 for Whisper widths).
// ------------------------------------------------------------------------------------------------
template <DT T, int MT, int NW>
__global__ __launch_bounds__(NW * 64) void gemm_skinny_kernel(const uint16_t* __restrict__ A, long lda,
                                                              const uint16_t* __restrict__ W, long ldw, int M, int N,
                                                              int K, Epi e) {
  // NW waves split K; each wave issues KU k-steps of loads (KU weight + KU*MT activation fragments) before any MFMA
  constexpr int KU = MT <= 2 ? 8 : (MT <= 4 ? 4 : (MT <= 8 ? 2 : 1));
  constexpr int LDR = 17;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [NW][MT*16][LDR]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int n = min(n0 + fr, N - 1);
  const int ksteps = K / 32;
  const int per = (ksteps + NW - 1) / NW;
  const int ks0 = wave * per, ks1 = min(ksteps, ks0 + per);
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0, 0, 0, 0};
  const uint16_t* wrow = W + (long)n * ldw + 8 * fq;
  // rows >= M are clamped to M-1: they only feed output rows that are never stored
  const uint16_t* arow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) arow[i] = A + (long)min(i * 16 + fr, M - 1) * lda + 8 * fq;
  for (int kk = ks0; kk < ks1; kk += KU) {
    u16x8 b[KU], av[KU][MT];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int k = min(kk + u, ks1 - 1) * 32;
      b[u] = *reinterpret_cast<const u16x8*>(wrow + k);
#pragma unroll
      for (int i = 0; i < MT; ++i) av[u][i] = *reinterpret_cast<const u16x8*>(arow[i] + k);
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (kk + u < ks1) {
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = mfma16<T>(av[u][i], b[u], acc[i]);
      }
    }
  }
  // every wave parks its partial tile (lane: rows i*16 + fq*4 + r, column fr); then all threads sum over waves
  float* mine = red + (long)wave * MT * 16 * LDR;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) mine[(i * 16 + fq * 4 + r) * LDR + fr] = acc[i][r];
  __syncthreads();
  // epilogue: 4 columns per thread
  for (int idx = tid; idx < MT * 16 * 4; idx += NW * 64) {
    const int row = idx >> 2, c4 = (idx & 3) * 4;
    const int m = row, nn = n0 + c4;
    if (m >= M || nn >= N) continue;
    float v4[4] = {0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < NW; ++w) {
      const float* p = red + ((long)w * MT * 16 + row) * LDR + c4;
#pragma unroll
      for (int q = 0; q < 4; ++q) v4[q] += p[q];
    }
    const float4 v = make_float4(v4[0], v4[1], v4[2], v4[3]);
    if (nn + 3 < N && (e.ldc & 3) == 0) {
      epi_store4<T>(e, m, nn, v);
    } else {
      for (int q = 0; q < 4 && nn + q < N; ++q) epi_store<T>(e, m, nn + q, v4[q]);
    }
  }
}

template <DT T, int MT, int NW>
static void launch_skinny_cfg(const GemmCall& g, hipStream_t st) {
  const size_t smem = (size_t)NW * MT * 16 * 17 * sizeof(float);
  hipLaunchKernelGGL((gemm_skinny_kernel<T, MT, NW>), dim3((g.N + 15) / 16), dim3(NW * 64), smem, st, g.A, g.lda, g.W,
                     g.ldw, g.M, g.N, g.K, g.epi);
}

template <DT T, int MT, int NW>
static void skinny_attr() {
  const size_t smem = (size_t)NW * MT * 16 * 17 * sizeof(float);
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_skinny_kernel<T, MT, NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)smem));
}

// set every kernel attribute up front (never inside a stream capture)
template <DT T>
static void g256_attr();

void gemm_init_attributes() {
  static bool done = false;
  if (done) return;
  skinny_attr<DT::BF16, 1, 16>();
  skinny_attr<DT::BF16, 2, 16>();
  skinny_attr<DT::BF16, 4, 16>();
  skinny_attr<DT::BF16, 8, 8>();
  skinny_attr<DT::BF16, 12, 4>();
  skinny_attr<DT::BF16, 16, 4>();
  skinny_attr<DT::F16, 1, 16>();
  skinny_attr<DT::F16, 2, 16>();
  skinny_attr<DT::F16, 4, 16>();
  skinny_attr<DT::F16, 8, 8>();
  skinny_attr<DT::F16, 12, 4>();
  skinny_attr<DT::F16, 16, 4>();
  g256_attr<DT::BF16>();
  g256_attr<DT::F16>();
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_kernel<DT::BF16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kMx8Lds));
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_kernel<DT::F16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kMx8Lds));
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_256_kernel<DT::BF16, EPI_STORE16>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kMx8bLds));
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_256_kernel<DT::BF16, EPI_RESID32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kMx8bLds));
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_256_kernel<DT::BF16, EPI_GELU_MX8>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kMx8bLds));
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_256_kernel<DT::F16, EPI_STORE16>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kMx8bLds));
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_256_kernel<DT::F16, EPI_RESID32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kMx8bLds));
  WMX_HIP(hipFuncSetAttribute((const void*)gemm_mx8_256_kernel<DT::F16, EPI_GELU_MX8>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kMx8bLds));
  done = true;
}

template <DT T>
static void launch_skinny(const GemmCall& g, hipStream_t st) {
  WMX_CHECK(g.K % 32 == 0 && g.M <= 256, "skinny gemm: shape");
  const int mt = (g.M + 15) / 16;
  if (mt <= 1)
    launch_skinny_cfg<T, 1, 16>(g, st);
  else if (mt <= 2)
    launch_skinny_cfg<T, 2, 16>(g, st);
  else if (mt <= 4)
    launch_skinny_cfg<T, 4, 16>(g, st);
  else if (mt <= 8)
    launch_skinny_cfg<T, 8, 8>(g, st);
  else if (mt <= 12)
    launch_skinny_cfg<T, 12, 4>(g, st);
  else
    launch_skinny_cfg<T, 16, 4>(g, st);
}

// ------------------------------------------------------------------------------------------------
// decode GEMM on packed weights (skinny M): workgroup = NCT 16-column tiles x one K slice x one 16*MT row chunk;
// its 4 waves split the slice's k-steps, every wave issues KU k-steps of loads (NCT contiguous 1 KiB weight
// fragments + MT activation fragments) before their MFMAs, partial tiles are summed through LDS.
// Grid (col groups, S, row chunks).  S == 1: epilogue; S > 1: raw fp32 partials part[s][M][N].
// ------------------------------------------------------------------------------------------------
// k-steps per load batch.  The loads of a batch are unconditional (k-step index clamped to the wave's last one;
// only the MFMAs are guarded): with per-step guarded loads, 4 k-steps per batch faulted with an illegal address in
// the micro decode although every guarded address is in bounds (tests/test_packed_extent.py) -- the clamped form
// is straight-line code.  The unsplit residual producers (MT + NCT <= 3, fc2: 10 k-steps per wave) take 5 per batch.
template <int MT, int NCT>
constexpr int packed_ku() {
  return (MT + NCT) <= 3 ? 5 : (MT + NCT) <= 8 ? 2 : 1;
}
// 8-bit weights: a k-step is 64 deep (one 16-byte weight piece + two A fragments per 16-row tile); the waves per
// workgroup come from the 32-deep step count as for 16-bit weights (packed_nw), so a wave holds 1-2 of these wider
// k-steps and issues them as one batch
template <int MT, int NCT>
constexpr int packed_ku8() {
  return (MT + NCT) <= 3 ? 3 : (MT + NCT) <= 8 ? 2 : 1;
}

// S == 1 epilogues of the LayerNorm-folded decode step (wmx_common.h row_ln_from_stats): the residual producer
// (x += acc + bias, its 16-bit copy and per-16-column statistics) and the folded-LN + GELU consumer (fc1).
// Trip counts are whole waves (MT * 16 * 4 NCT is a multiple of 64), so the 4-lane DPP sums see every lane.
// The consumer's row statistics and the producer's residual quad are loaded before the main loop (FoldPre, beside
// the first weight batch), so neither is a round trip after the reduction barrier.
template <int MT, int NW>
struct FoldPre {
  static constexpr int RPW = (MT * 16 + NW - 1) / NW;  // statistics rows per wave (rows wave + NW j)
  static constexpr int RPH = (RPW + 1) / 2;              // row pairs: rows wave + NW 2p (lanes 0..31), + NW (2p + 1)
  float2 s[RPH][4];
  // EPI_RESID_STATS: q0 = the residual quad of this thread's first epilogue item (idx = tid); EPI_LNFOLD_GELU16:
  // q0 / q1 = the folded constants c1 / c2 of the thread's column quad (the same in every row).  One slot for both
  // kinds, each assigned whole: two members loaded on either side of a branch were merged into one load stored
  // through a selected pointer, which demoted the whole struct to scratch in every generic instantiation
  float4 q0, q1;
};
template <DT T, int MT, int NCT, int NW, bool LNF>
__device__ __forceinline__ void packed_fold_prefetch(FoldPre<MT, NW>& P, const Epi& e, int M, int N, int K, int m0,
                                                     int t0) {
  constexpr int C4 = 4 * NCT;
  const int tid = threadIdx.x, wave = tid >> 6;
  if constexpr (LNF) {
#pragma unroll
    for (int p = 0; p < FoldPre<MT, NW>::RPH; ++p) {
      const long ra = min(m0 + min(wave + NW * 2 * p, MT * 16 - 1), M - 1);
      const long rb = min(m0 + min(wave + NW * (2 * p + 1), MT * 16 - 1), M - 1);
      row_ln_stats_load2(e.stats + ra * e.stats_ld, e.stats + rb * e.stats_ld, K >> 4, P.s[p]);
    }
    const int n = min(t0 * 16 + (tid % C4) * 4, N - 4);
    P.q0 = *reinterpret_cast<const float4*>(e.c1 + n);
    P.q1 = *reinterpret_cast<const float4*>(e.c2 + n);
  } else {
    const int row = tid / C4, c = (tid - row * C4) * 4;
    const int m = min(m0 + min(row, MT * 16 - 1), M - 1), n = min(t0 * 16 + c, N - 4);
    P.q0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(e.out) + (long)m * e.ldc + n);
    P.q1 = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
// the LayerNorm-folded consumer's merged (mean, rstd) of its rows, in LDS
template <int MT>
__device__ __forceinline__ float2* fold_rln() {
  __shared__ float2 r[MT * 16];
  return r;
}
// merged while the wave's first weight batch is in flight (the statistics loads were issued before it), so the
// epilogue needs no merge and no barrier of its own: the reduction barrier orders these LDS writes before its reads
template <int MT, int NW>
__device__ __forceinline__ void packed_fold_merge(const FoldPre<MT, NW>& P, int K) {
  const int tid = threadIdx.x, wave = tid >> 6;
  float2* rln = fold_rln<MT>();
#pragma unroll
  for (int p = 0; p < FoldPre<MT, NW>::RPH; ++p) {
    const int r = wave + NW * (2 * p + ((tid & 63) >> 5));  // this half-wave's row
    const float2 st = row_ln_stats_merge2(P.s[p], K >> 4);
    if ((tid & 31) == 0 && r < MT * 16) rln[r] = st;
  }
}
template <DT T, int MT, int NCT, int NW, bool LNF>
__device__ __forceinline__ void packed_fold_epilogue(const float (&red)[NW][MT * 16][16 * NCT + 1], const Epi& e,
                                                     int M, int N, int K, int m0, int t0, const FoldPre<MT, NW>& P) {
  constexpr int NT = 64 * NW, C4 = 4 * NCT;
  const int tid = threadIdx.x, wave = tid >> 6;
  constexpr bool fold = LNF;
  const float2* rln = fold ? fold_rln<MT>() : nullptr;  // (merged by packed_fold_merge before the reduction barrier)
  for (int idx = tid; idx < MT * 16 * C4; idx += NT) {
    const int row = idx / C4, c = (idx - row * C4) * 4;
    const int m = m0 + row, n = t0 * 16 + c;
    const bool ok = m < M && n < N;
    float v4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = red[0][row][c + q];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += red[w][row][c + q];
      v4[q] = v;
    }
    if constexpr (!fold) {
      float* xp = reinterpret_cast<float*>(e.out) + (long)m * e.ldc + n;
      const float4 x0 = idx == tid ? P.q0 : ok ? *reinterpret_cast<const float4*>(xp) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 b = ok && e.bias ? *reinterpret_cast<const float4*>(e.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
      // the order of the split-K path: x + bias + sum (reduce_ln4_kernel)
      const float4 x = make_float4(x0.x + b.x + v4[0], x0.y + b.y + v4[1], x0.z + b.z + v4[2], x0.w + b.w + v4[3]);
      const float mean = sum4_lanes((x.x + x.y) + (x.z + x.w)) * (1.f / 16.f);
      const float dx = x.x - mean, dy = x.y - mean, dz = x.z - mean, dw = x.w - mean;
      const float m2 = sum4_lanes((dx * dx + dy * dy) + (dz * dz + dw * dw));
      if (ok) {
        *reinterpret_cast<float4*>(xp) = x;
        const u16x4 h = {from_f32<T>(x.x), from_f32<T>(x.y), from_f32<T>(x.z), from_f32<T>(x.w)};
        *reinterpret_cast<u16x4*>(e.out16 + (long)m * e.ldc + n) = h;
        if ((n & 15) == 0) e.stats[(long)m * e.stats_ld + (n >> 4)] = make_float2(mean, m2);  // [R][d / 16]
      }
    } else {
      if (!ok) continue;
      const float2 ln = rln[row];
      const float4 a = P.q0, b = P.q1;  // (prefetched: a thread's column quad is the same in every row, NT % C4 == 0)
      const u16x4 h = {from_f32<T>(gelu_erf(ln.y * (v4[0] - ln.x * a.x) + b.x)),
                       from_f32<T>(gelu_erf(ln.y * (v4[1] - ln.x * a.y) + b.y)),
                       from_f32<T>(gelu_erf(ln.y * (v4[2] - ln.x * a.z) + b.z)),
                       from_f32<T>(gelu_erf(ln.y * (v4[3] - ln.x * a.w) + b.w))};
      *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + (long)m * e.ldc + n) = h;
    }
  }
}

// Epilogue class, a template parameter so each launch carries only the code it runs (these launches are a few
// microseconds long and start on a cold instruction cache: a generic epilogue switch in a split-K launch measured
// +0.6 us per launch): kPackedPart split-K raw partials (S > 1); kPackedGelu S == 1 bias + GELU -> 16-bit
// (decode fc1; bias loaded beside the first k-steps); kPackedResidStats / kPackedLnfGelu the mixed step's folded
// LayerNorm producer / consumer (round 6: their own instantiations, no longer branches of the generic one);
// kPackedGeneric every other S == 1 epilogue
enum { kPackedPart = 0, kPackedGelu = 1, kPackedGeneric = 2, kPackedResidStats = 3, kPackedLnfGelu = 4 };

// W8: the weights are e4m3 bytes in the packed8_index layout with per-row scales wsc (a k-step is 64 deep: the
// same 16-byte lane load as a bf16 k-step, widened in registers into the B fragments of two MFMAs; the row scale
// multiplies the reduced fp32 tile before any epilogue or partial store)
template <DT T, int MT, int NCT, int NW, int EPK, int W8 = 0>
__global__ __launch_bounds__(64 * NW) void gemm_packed_kernel(const uint16_t* __restrict__ A, long lda,
                                                              const uint16_t* __restrict__ Wp, int M, int N, int K,
                                                              int S, Epi e, float* __restrict__ part,
                                                              unsigned long long* __restrict__ tprobe,
                                                              const int* __restrict__ pslot,
                                                              const float* __restrict__ wsc) {
  constexpr int KU = W8 ? packed_ku8<MT, NCT>() : packed_ku<MT, NCT>();
  constexpr int LDR = 16 * NCT + 1;
  constexpr int NT = 64 * NW;
  __shared__ float red[NW][MT * 16][LDR];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  // in-situ probe (bench roofline): this workgroup's start / end, device wall-clock ticks
  const unsigned long long probe_t0 = (tprobe && tid == 0) ? probe_clock() : 0ull;
  const int ntiles = (N + 15) >> 4;
  const int t0 = blockIdx.x * NCT;
  const int sp = blockIdx.y;
  const int m0 = blockIdx.z * MT * 16;
  const int ksteps = W8 ? K >> 6 : K >> 5;
  int ks0, ks1;
  packed_wave_ksteps(W8 ? K >> 1 : K, S, NW, sp, wave, ks0, ks1);
  // kPackedGelu: a thread's column quad is the same in every row it stores (NT is a multiple of 4 NCT), so its
  // bias is loaded now, beside the first k-step batch, not as a round trip after the reduction barrier (the 8-bit
  // row scales likewise; the scale array is padded to whole 16-row tiles)
  float4 pbias = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (EPK == kPackedGelu)
    pbias = *reinterpret_cast<const float4*>(e.bias + min(t0 * 16 + (tid % (4 * NCT)) * 4, N - 4));
  float4 wsc4 = make_float4(1.f, 1.f, 1.f, 1.f);
  if constexpr (W8) wsc4 = *reinterpret_cast<const float4*>(wsc + min(t0 * 16 + (tid % (4 * NCT)) * 4, ntiles * 16 - 4));
  // the folded-LayerNorm epilogues (S == 1): their statistics / residual loads ride ahead of the main loop
  constexpr bool fold_epi = (EPK == kPackedResidStats || EPK == kPackedLnfGelu) && !W8;  // (S == 1: host-checked)
  FoldPre<MT, NW> fpre;
  if constexpr (fold_epi) packed_fold_prefetch<T, MT, NCT, NW, EPK == kPackedLnfGelu>(fpre, e, M, N, K, m0, t0);
  f32x4 acc[MT][NCT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  const uint16_t* wt[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) wt[j] = Wp + packed_w_elem(t0 + j, ntiles, ksteps, 0, lane);
  // rows >= M are clamped to M-1: they only feed output rows that are never stored
  const uint16_t* ar[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) ar[i] = A + packed_a_elem(m0 + i * 16 + fr, M, lda, 0, lane);
  if constexpr (W8) {
    for (int kk = ks0; kk < ks1; kk += KU) {
      u32x4 b[KU][NCT];
      u16x8 av[KU][MT][2];
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int k = min(kk + u, ks1 - 1);  // clamped: a duplicate load of the wave's last k-step, MFMA skipped
#pragma unroll
        for (int j = 0; j < NCT; ++j) b[u][j] = stream_load(reinterpret_cast<const u32x4*>(wt[j] + ((long)k << 9)));
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          av[u][i][0] = *reinterpret_cast<const u16x8*>(ar[i] + k * 64);
          av[u][i][1] = *reinterpret_cast<const u16x8*>(ar[i] + k * 64 + 32);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < KU; ++u)
        if (kk + u < ks1)
#pragma unroll
          for (int j = 0; j < NCT; ++j) {
            u16x8 blo, bhi;
            if constexpr (W8 == 2)
              i8x16_to16<T>(b[u][j], blo, bhi);
            else
              fp8x16_to16<T>(b[u][j], blo, bhi);
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              acc[i][j] = mfma16<T>(av[u][i][0], blo, acc[i][j]);
              acc[i][j] = mfma16<T>(av[u][i][1], bhi, acc[i][j]);
            }
          }
    }
  }
  bool merged = false;  // (LNF: wave-uniform)
  for (int kk = ks0; !W8 && kk < ks1; kk += KU) {
    u16x8 b[KU][NCT], av[KU][MT];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int k = min(kk + u, ks1 - 1);  // clamped: a duplicate load of the wave's last k-step, MFMA skipped
#pragma unroll
      for (int j = 0; j < NCT; ++j) b[u][j] = stream_load(reinterpret_cast<const u16x8*>(wt[j] + ((long)k << 9)));
#pragma unroll
      for (int i = 0; i < MT; ++i) av[u][i] = *reinterpret_cast<const u16x8*>(ar[i] + k * 32);
    }
    // the whole batch is in flight before the first MFMA: without this fence the scheduler may interleave a
    // load behind an MFMA and wait for it with vmcnt(0), two round trips per batch instead of one (measured +1 us
    // per split-K launch in one instantiation)
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (EPK == kPackedLnfGelu && !W8) {
      if (!merged) {
        packed_fold_merge<MT, NW>(fpre, K);
        merged = true;
      }
    }
#pragma unroll
    for (int u = 0; u < KU; ++u)
      if (kk + u < ks1)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NCT; ++j) acc[i][j] = mfma16<T>(av[u][i], b[u][j], acc[i][j]);
  }
  if constexpr (EPK == kPackedLnfGelu && !W8)
    if (!merged) packed_fold_merge<MT, NW>(fpre, K);  // (a wave without k-steps)
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NCT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][i * 16 + fq * 4 + r][j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  // 4 consecutive columns per thread
  constexpr int C4 = 4 * NCT;  // column quads per row
  if constexpr (fold_epi)  // (the folded step has no 8-bit form: host-checked)
    packed_fold_epilogue<T, MT, NCT, NW, EPK == kPackedLnfGelu>(red, e, M, N, K, m0, t0, fpre);
  for (int idx = tid; !fold_epi && idx < MT * 16 * C4; idx += NT) {
    const int row = idx / C4, c = (idx - row * C4) * 4;
    const int m = m0 + row, n = t0 * 16 + c;
    if (m >= M || n >= N) continue;
    float v4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = red[0][row][c + q];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += red[w][row][c + q];
      v4[q] = v;
    }
    if constexpr (W8) {
      v4[0] *= wsc4.x;
      v4[1] *= wsc4.y;
      v4[2] *= wsc4.z;
      v4[3] *= wsc4.w;
    }
    if constexpr (EPK == kPackedGelu) {  // N and ldc multiples of 4 (host-checked)
      const u16x4 h = {from_f32<T>(gelu_erf(v4[0] + pbias.x)), from_f32<T>(gelu_erf(v4[1] + pbias.y)),
                       from_f32<T>(gelu_erf(v4[2] + pbias.z)), from_f32<T>(gelu_erf(v4[3] + pbias.w))};
      *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(e.out) + (long)m * e.ldc + n) = h;
    } else if (EPK == kPackedPart || S > 1) {
      float* dst = part + ((long)sp * M + m) * N + n;
      if (n + 3 < N && (N & 3) == 0) {
        *reinterpret_cast<float4*>(dst) = make_float4(v4[0], v4[1], v4[2], v4[3]);
      } else {
        for (int q = 0; q < 4 && n + q < N; ++q) dst[q] = v4[q];
      }
    } else if constexpr (EPK == kPackedGeneric) {
      if (n + 3 < N && (e.ldc & 3) == 0) {
        epi_store4<T>(e, m, n, make_float4(v4[0], v4[1], v4[2], v4[3]));
      } else {
        for (int q = 0; q < 4 && n + q < N; ++q) epi_store<T>(e, m, n + q, v4[q]);
      }
    }
  }
  if (tprobe && tid == 0) probe_record(tprobe, *pslot, probe_t0);
}

static int packed_mt(int M) {
  const int mt = (std::min(M, 128) + 15) / 16;
  return mt <= 4 ? mt : (mt <= 6 ? 6 : 4);
}

int packed_nct(int M, int N, int K) {
  const int mt = packed_mt(M);
  if (mt > 4) return 2;
  return (N >= 16384 || K >= 4096) ? 4 : 2;
}

int packed_splits(int M, int N, int K, long cap_elems) {
  const int mt = packed_mt(M);
  const int chunks = (M + mt * 16 - 1) / (mt * 16);
  const int nct = packed_nct(M, N, K);
  const long wgs = (long)((N + 16 * nct - 1) / (16 * nct)) * chunks;
  // workgroups a split aims for: 160 up to 24 rows (the bench's two groups of 4 windows x beam 5 decode in step, so
  // two launches of this size run at once; fewer slices = fewer partials for the consumers: 414.3-414.7x against
  // 410.5-410.8x with 480, profiles/r04_split_target/), 480 above (16 windows: 724.6 / 568.0x against 723.1 / 562.6x
  // with 240)
  const long target = M <= 24 ? 160L : 480L;
  long S = (target + wgs - 1) / wgs;
  S = std::min<long>(S, std::max(1, (K / 32) / 4));
  S = std::min<long>(S, K / (2L * std::max(M, 1)));
  S = std::min<long>(S, 8);  // the consumers load every slice of a value in one batch (reduce_ln: kRedMaxS)
  while (S > 1 && S * M * (long)N > cap_elems) --S;
  return (int)std::max<long>(1, S);
}

// waves per workgroup: enough that each wave's share of its K slice is at most ~4 k-steps (two dependent load
// batches), so long unsplit slices (fc1, whose GELU epilogue needs S = 1) are not a chain of five round trips
// the cross-wave reduction image red[NW][MT * 16][16 NCT + 1] of a workgroup: within 80 KiB (two workgroups per
// CU) always; up to the CU's 160 KiB when the launch has no more workgroups than the chip has CUs (one each anyway:
// R = 40's fc1 / fc2, MT 3 x NCT 4, whose 4 waves otherwise walk 5 / 3 dependent load batches)
template <int MT, int NCT>
constexpr int packed_red_bytes(int nw) { return nw * MT * 16 * (16 * NCT + 1) * 4; }
constexpr int kPackedOneWgPerCu = 256;

// (w8: the 8-bit decode keeps the 80 KiB budget: with the two groups in step, 8 waves on 8-bit weights measured
// 728.8-731.8x against 726.0-726.7x at 16 windows, while the 16-bit decode keeps its 16-wave fc2: 568.3 / 569.4x against
// 564.4 / 564.5x, profiles/r04_lds_budget/)
template <int MT, int NCT>
static int packed_nw(int K, int S, long wgs = 1L << 30, bool w8 = false) {
  const int ksteps = K / 32, kps = (ksteps + S - 1) / S;
  // k-steps per wave the wave count aims for: 4 (two dependent load batches; 2, 3 measured within noise, round 4)
  const int per4 = (kps + 3) / 4;
  const int budget = (!w8 && wgs <= kPackedOneWgPerCu) ? 163840 : 81920;
  const bool fit8 = packed_red_bytes<MT, NCT>(8) <= budget;
  const bool fit16 = packed_red_bytes<MT, NCT>(16) <= budget;
  if (per4 <= 4 || !fit8) return 4;
  if (per4 <= 8 || !fit16) return 8;
  return 16;
}

template <DT T, int MT, int NCT, int W8>
static void launch_packed_cfg(const PackedCall& g, hipStream_t st) {
  const int ntiles = (g.N + 15) / 16;
  dim3 grid((ntiles + NCT - 1) / NCT, g.S, (g.M + MT * 16 - 1) / (MT * 16));
  const int nw = packed_nw<MT, NCT>(g.K, g.S, (long)grid.x * grid.y * grid.z, W8 != 0);
  const int epk = g.S > 1 ? kPackedPart
                 : (g.epi.kind == EPI_GELU16 && g.epi.bias && g.N % 4 == 0 && g.epi.ldc % 4 == 0) ? kPackedGelu
                 : g.epi.kind == EPI_RESID_STATS ? kPackedResidStats
                 : g.epi.kind == EPI_LNFOLD_GELU16 ? kPackedLnfGelu
                                                   : kPackedGeneric;
#define WMX_PACKED_EPK(NWV, EPKV)                                                                                  \
  hipLaunchKernelGGL((gemm_packed_kernel<T, MT, NCT, NWV, EPKV, W8>), grid, dim3(64 * NWV), 0, st, g.A, g.lda, g.W,  \
                     g.M, g.N, g.K, g.S, g.epi, g.part, g.tprobe, g.pslot, g.wscale)
#define WMX_PACKED_LAUNCH(NWV)                                                                                     \
  do {                                                                                                             \
    switch (epk) {                                                                                                 \
      case kPackedPart: WMX_PACKED_EPK(NWV, kPackedPart); break;                                                   \
      case kPackedGelu: WMX_PACKED_EPK(NWV, kPackedGelu); break;                                                   \
      case kPackedResidStats:                                                                                      \
        if constexpr (W8 == 0) WMX_PACKED_EPK(NWV, kPackedResidStats);                                             \
        break;                                                                                                     \
      case kPackedLnfGelu:                                                                                         \
        if constexpr (W8 == 0) WMX_PACKED_EPK(NWV, kPackedLnfGelu);                                                \
        break;                                                                                                     \
      default: WMX_PACKED_EPK(NWV, kPackedGeneric); break;                                                         \
    }                                                                                                              \
  } while (0)
  constexpr bool fit8 = packed_red_bytes<MT, NCT>(8) <= 163840;
  constexpr bool fit16 = packed_red_bytes<MT, NCT>(16) <= 163840;
  if (nw == 4) {
    WMX_PACKED_LAUNCH(4);
  } else if (nw == 8) {
    if constexpr (fit8) WMX_PACKED_LAUNCH(8);
  } else {
    if constexpr (fit16) WMX_PACKED_LAUNCH(16);
  }
#undef WMX_PACKED_LAUNCH
#undef WMX_PACKED_EPK
}

template <int MT, int NCT>
static PackedPlan plan_cfg(int M, int N, int K, int S, bool w8) {
  const int gx = ((N + 15) / 16 + NCT - 1) / NCT, gz = (M + MT * 16 - 1) / (MT * 16);
  return PackedPlan{MT, NCT, packed_nw<MT, NCT>(K, S, (long)gx * S * gz, w8), w8 ? packed_ku8<MT, NCT>() : packed_ku<MT, NCT>(),
                    gx, gz};
}

template <int NCT>
static PackedPlan plan_mt(int M, int N, int K, int S, bool w8) {
  switch ((std::min(M, 128) + 15) / 16) {  // launch_packed_mt's dispatch
    case 1: return plan_cfg<1, NCT>(M, N, K, S, w8);
    case 2: return plan_cfg<2, NCT>(M, N, K, S, w8);
    case 3: return plan_cfg<3, NCT>(M, N, K, S, w8);
    case 4: return plan_cfg<4, NCT>(M, N, K, S, w8);
    case 5:
    case 6: return plan_cfg<6, 2>(M, N, K, S, w8);
    default: return plan_cfg<4, 2>(M, N, K, S, w8);
  }
}

PackedPlan packed_plan(int M, int N, int K, int S, int nct, bool w8) {
  const int c = nct ? nct : packed_nct(M, N, K);
  return c == 4 ? plan_mt<4>(M, N, K, S, w8) : c == 1 ? plan_mt<1>(M, N, K, S, w8) : plan_mt<2>(M, N, K, S, w8);
}

// walks every lane of every wave of every workgroup of the launch through the kernel's own index helpers
// (w8: w_end in BYTES of the packed8 weights, k-steps 64 deep reading A fragments 2k and 2k + 1)
PackedExtent packed_extent(int M, int N, int K, int S, long lda, int nct, bool w8) {
  const PackedPlan p = packed_plan(M, N, K, S, nct, w8);
  const int ntiles = (N + 15) / 16, ksteps = w8 ? K / 64 : K / 32;
  PackedExtent e{0, 0, 0, 0};
  for (int bx = 0; bx < p.gx; ++bx)
    for (int sp = 0; sp < S; ++sp)
      for (int bz = 0; bz < p.gz; ++bz)
        for (int wave = 0; wave < p.NW; ++wave) {
          int ks0, ks1;
          packed_wave_ksteps(w8 ? K / 2 : K, S, p.NW, sp, wave, ks0, ks1);
          for (int kk = ks0; kk < ks1; kk += p.KU)
            for (int u = 0; u < p.KU; ++u) {
              const int k = std::min(kk + u, ks1 - 1);  // the kernel's clamped load index
              if (k < 0 || k >= ksteps) ++e.stray_ksteps;
              // both offsets grow with the lane index (lane * 8; row lane & 15 and column 8 * (lane >> 4)), so
              // lane 63 bounds the wave
              for (int lane = 63; lane < 64; lane += 1) {
                for (int j = 0; j < p.NCT; ++j)
                  e.w_end = std::max(e.w_end, w8 ? 2 * packed_w_elem(bx * p.NCT + j, ntiles, ksteps, k, lane) + 16
                                                 : packed_w_elem(bx * p.NCT + j, ntiles, ksteps, k, lane) + 8);
                for (int i = 0; i < p.MT; ++i)
                  e.a_end = std::max(e.a_end, packed_a_elem(bz * p.MT * 16 + i * 16 + (lane & 15), M, lda,
                                                            w8 ? 2 * k + 1 : k, lane) + 8);
              }
            }
          if (S > 1)  // partial stores: rows < M, column quads < N
            for (int row = 0; row < p.MT * 16; ++row)
              for (int c = 0; c < 16 * p.NCT; c += 4) {
                const int m = bz * p.MT * 16 + row, n = bx * p.NCT * 16 + c;
                if (m < M && n < N) e.part_end = std::max(e.part_end, ((long)sp * M + m) * N + std::min(n + 4, N));
              }
        }
  return e;
}

template <DT T, int NCT, int W8>
static void launch_packed_mt(const PackedCall& g, hipStream_t st) {
  const int mt = (std::min(g.M, 128) + 15) / 16;
  switch (mt) {
    case 1: launch_packed_cfg<T, 1, NCT, W8>(g, st); break;
    case 2: launch_packed_cfg<T, 2, NCT, W8>(g, st); break;
    case 3: launch_packed_cfg<T, 3, NCT, W8>(g, st); break;
    case 4: launch_packed_cfg<T, 4, NCT, W8>(g, st); break;
    case 5:
    case 6: launch_packed_cfg<T, 6, 2, W8>(g, st); break;
    default: launch_packed_cfg<T, 4, 2, W8>(g, st); break;  // 7..8 row tiles: 64-row chunks (LDS budget)
  }
}
template <DT T, int W8>
static void launch_packed_nct(int nct, const PackedCall& g, hipStream_t st) {
  if (nct == 4) launch_packed_mt<T, 4, W8>(g, st);
  else if (nct == 1) launch_packed_mt<T, 1, W8>(g, st);
  else launch_packed_mt<T, 2, W8>(g, st);
}

void launch_gemm_packed(DT dt, const PackedCall& g, hipStream_t st) {
  WMX_CHECK(g.M >= 1 && g.K % 32 == 0 && g.S >= 1, "packed gemm: shape");
  WMX_CHECK(g.S == 1 || g.part != nullptr, "packed gemm: partial buffer required for S > 1");
  WMX_CHECK(g.nct == 0 || g.nct == 1 || g.nct == 2 || g.nct == 4, "packed gemm: column tiles per workgroup");
  WMX_CHECK((g.epi.kind != EPI_RESID_STATS && g.epi.kind != EPI_LNFOLD_GELU16) ||
                (g.S == 1 && g.N % 16 == 0 && g.epi.stats && g.epi.ldc % 4 == 0 &&
                 (g.epi.kind == EPI_LNFOLD_GELU16
                      ? (g.epi.c1 && g.epi.c2 && g.K % 16 == 0 && g.K <= 2048 && g.epi.stats_ld >= g.K / 16)
                      : (g.epi.out16 != nullptr && g.N <= 2048 && g.epi.stats_ld >= g.N / 16))),
            "packed gemm: folded-LayerNorm epilogue arguments");
  const bool w8 = g.wscale != nullptr;
  WMX_CHECK(!w8 || (g.K % 64 == 0 && g.epi.kind != EPI_RESID_STATS && g.epi.kind != EPI_LNFOLD_GELU16),
            "packed gemm: 8-bit weights need K % 64 == 0 and no folded-LayerNorm epilogue");
  const int nct = g.nct ? g.nct : packed_nct(g.M, g.N, g.K);
  // (8-bit weights: e4m3 bytes (w8kind 1, the fp8 decode) or int8 bytes (w8kind 2, the CTranslate2 int8 grid))
  const int kind = w8 ? (g.w8kind == 2 ? 2 : 1) : 0;
  if (dt == DT::BF16) {
    if (kind == 2) launch_packed_nct<DT::BF16, 2>(nct, g, st);
    else if (kind == 1) launch_packed_nct<DT::BF16, 1>(nct, g, st);
    else launch_packed_nct<DT::BF16, 0>(nct, g, st);
  } else {
    if (kind == 2) launch_packed_nct<DT::F16, 2>(nct, g, st);
    else if (kind == 1) launch_packed_nct<DT::F16, 1>(nct, g, st);
    else launch_packed_nct<DT::F16, 0>(nct, g, st);
  }
  WMX_HIP(hipGetLastError());
}


template <DT T, int BM, int BN, int WM, int WN>
static void launch_cfg(const GemmCall& g, hipStream_t st) {
  constexpr int TILE_BYTES = (BM + BN) * 128;
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  int splits = std::max(1, g.splits);
  int kchunk = ((g.K / 64 + splits - 1) / splits) * 64;
  splits = (g.K + kchunk - 1) / kchunk;
  float* ws = splits > 1 ? g.ws : nullptr;
  if (splits > 1) WMX_CHECK(ws != nullptr && (long)splits * g.M * g.N <= g.ws_elems, "gemm: split-K workspace too small");
  dim3 grid(tiles, splits);
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN>), grid, dim3(WM * WN * 64), 2 * TILE_BYTES, st, g.A, g.lda, g.W,
                     g.ldw, g.M, g.N, g.K, kchunk, g.epi, ws);
  if (splits > 1) {
    long total = (long)g.M * g.N;
    int blocks = (int)std::min<long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL((gemm_splitk_reduce<T>), dim3(blocks), dim3(256), 0, st, g.ws, splits, g.M, g.N, g.epi);
  }
}

// gemm256 instantiations: one per vectorisable epilogue kind (the epilogue's registers then hold only what that
// kind needs), plus the generic one (-1) for the cross-K/V scatter and unaligned outputs
template <DT T, int KIND>
static void g256_attr_one() {
  WMX_HIP(hipFuncSetAttribute((const void*)gemm256_kernel<T, KIND>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              g256_lds<KIND>()));
}
template <DT T>
static void g256_attr() {
  g256_attr_one<T, -1>();
  g256_attr_one<T, EPI_STORE16>();
  g256_attr_one<T, EPI_GELU16>();
  g256_attr_one<T, EPI_RESID32>();
  g256_attr_one<T, EPI_GELU_POS32>();
  g256_attr_one<T, EPI_STORE32>();
  g256_attr_one<T, EPI_GELU_MX8>();
  g256_attr_one<T, EPI_CROSSKV>();
  g256_attr_one<T, EPI_RESID32_LNS>();
  g256_attr_one<T, EPI_GELU_POS32_LNS>();
  g256_attr_one<T, EPI_LNF_STORE16>();
  g256_attr_one<T, EPI_LNF_GELU16>();
}
// persistent grid: one workgroup per CU (the 128 KiB ring allows no second one), a multiple of 8 workgroups
static int g256_grid(int tiles) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess)
      n = 256;
    return std::max(8, n / 8 * 8);
  }();
  return std::min(tiles, cus);
}

template <DT T>
static void launch_g256(const GemmCall& g, hipStream_t st) {
  const int ntile = ((g.M + 255) / 256) * ((g.N + 255) / 256);
  const int tiles = g256_grid(ntile);
  const bool vec = (g.N & 3) == 0 && (g.epi.ldc & 3) == 0;
  const int kind = (vec || g.epi.kind == EPI_CROSSKV) ? g.epi.kind : -1;
#define WMX_G256_LAUNCH(KD)                                                                                    \
  hipLaunchKernelGGL((gemm256_kernel<T, KD>), dim3(tiles), dim3(512), g256_lds<KD>(), st, g.A, g.lda, g.W, g.ldw, g.M, \
                     g.N, g.K, g.epi)
  switch (kind) {
    case EPI_STORE16: WMX_G256_LAUNCH(EPI_STORE16); break;
    case EPI_GELU16: WMX_G256_LAUNCH(EPI_GELU16); break;
    case EPI_RESID32: WMX_G256_LAUNCH(EPI_RESID32); break;
    case EPI_GELU_POS32: WMX_G256_LAUNCH(EPI_GELU_POS32); break;
    case EPI_STORE32: WMX_G256_LAUNCH(EPI_STORE32); break;
    case EPI_GELU_MX8: WMX_G256_LAUNCH(EPI_GELU_MX8); break;
    case EPI_CROSSKV: WMX_G256_LAUNCH(EPI_CROSSKV); break;
    case EPI_RESID32_LNS: WMX_G256_LAUNCH(EPI_RESID32_LNS); break;
    case EPI_GELU_POS32_LNS: WMX_G256_LAUNCH(EPI_GELU_POS32_LNS); break;
    case EPI_LNF_STORE16: WMX_G256_LAUNCH(EPI_LNF_STORE16); break;
    case EPI_LNF_GELU16: WMX_G256_LAUNCH(EPI_LNF_GELU16); break;
    default: WMX_G256_LAUNCH(-1); break;
  }
#undef WMX_G256_LAUNCH
}

template <DT T>
static void launch_t(const GemmCall& g, hipStream_t st) {
  if (g.tile == TILE_SKINNY) {
    launch_skinny<T>(g, st);
    return;
  }
  if (g.tile == TILE_256) {
    WMX_CHECK(g.K % WMX_G256_BK == 0 && g.lda % 8 == 0 && g.ldw % 8 == 0, "gemm256: K / leading dimensions");
    // the ring's per-lane element offsets are 32-bit (m lda + chunk, n ldw + chunk; the K-tile offset is added as long)
    WMX_CHECK(g256_offsets_fit(g.M, g.N, g.lda, g.ldw), "gemm256: M x lda or N x ldw exceeds 32-bit element offsets");
    WMX_CHECK(g.epi.kind != EPI_CROSSKV || (g.epi.d % 256 == 0 && g.epi.xt % 4 == 0), "gemm256: cross K/V shape");
    const bool lns = g.epi.kind == EPI_RESID32_LNS || g.epi.kind == EPI_GELU_POS32_LNS;
    const bool lnf = g.epi.kind == EPI_LNF_STORE16 || g.epi.kind == EPI_LNF_GELU16;
    WMX_CHECK(!lns || (g.N % 256 == 0 && g.epi.ldc % 256 == 0 && g.epi.out16 && g.epi.stats && g.epi.stats_ld >= g.M),
              "gemm256: LayerNorm-statistics epilogue shape");
    // the consumer's statistics DMA reads 16-byte (mean, M2) pairs at rows min(m0 + 2 lane, M - 2): M and the
    // statistics stride even; the fold is LayerNorm over exactly the GEMM's K (lng groups of 256 columns)
    WMX_CHECK(!lnf || (g.N % 4 == 0 && g.epi.ldc % 4 == 0 && g.epi.c1 && g.epi.bias && g.epi.stats &&
                       g.epi.lng >= 1 && g.epi.lng <= 8 && g.epi.stats_ld >= g.M && g.M % 2 == 0 &&
                       g.epi.stats_ld % 2 == 0 && g.K == 256 * g.epi.lng),
              "gemm256: LayerNorm-folded epilogue shape");
    launch_g256<T>(g, st);
    return;
  }
  WMX_CHECK(g.K % 64 == 0, "gemm: K must be a multiple of 64");
  switch (g.tile) {
    case TILE_128x128:
      launch_cfg<T, 128, 128, 2, 2>(g, st);
      break;
    case TILE_64x64:
      launch_cfg<T, 64, 64, 2, 2>(g, st);
      break;
    case TILE_32x64:
      launch_cfg<T, 32, 64, 1, 4>(g, st);
      break;
    default:
      WMX_CHECK(false, "gemm: bad tile");
  }
}

void launch_gemm(DT dt, const GemmCall& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return;
  if (dt == DT::BF16)
    launch_t<DT::BF16>(g, st);
  else
    launch_t<DT::F16>(g, st);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
