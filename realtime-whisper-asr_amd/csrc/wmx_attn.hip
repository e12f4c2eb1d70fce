// Attention kernels (SURVEY.md §2a rows "Encoder MHA", "Decoder self-attn w/ KV cache", "Decoder cross-attn").
//
// attn_flash: non-causal (encoder, T=1500) or causal/prefix-masked (decoder prefill) flash attention on
//   v_mfma_f32_16x16x32.  Swapped product S^T = K.Q^T puts a query on the lane, so the softmax row lives
//   in-lane + 4 lane groups, and P^T feeds the P.V MFMA as its B operand with no LDS round trip
//   (the k-order inside a 32-key step is permuted identically on the V^T operand).  K tile is XOR-swizzled
//   for conflict-free ds_read_b128; V is transposed into a padded LDS image during staging.
// dec_self_attn: one wave per (row, head, new token); keys are gathered through the beam ancestry table
//   (row whose cache slot holds the history of row r), so beam reordering never copies the KV cache.
// dec_cross_attn: one workgroup per (window, head): all beams of a window share one streamed read of the
//   window's cross K/V (the dominant HBM stream of the decode loop).
#include <cstdlib>

#include "wmx_common.h"
#include "wmx_kernels.h"


namespace wmx {

constexpr float kLog2e = 1.4426950408889634f;

// ------------------------------------------------------------------------------------------------
// flash attention, head_dim 64
// ------------------------------------------------------------------------------------------------
struct FlashArgs {
  AttnArgs a;
  int causal;          // key index <= query index + causal_off
  int causal_off;
  const int* kbegin;   // [B] first valid key (left padding), nullable
};

template <DT T>
__global__ __launch_bounds__(256) void attn_flash_kernel(FlashArgs fa) {
  const AttnArgs& a = fa.a;
  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, fr = lane & 15;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[64 * 64];
  constexpr int VTLD = 68;
  __shared__ __attribute__((aligned(16))) uint16_t Vt[64 * VTLD];

  const uint16_t* qb = a.q + (long)b * a.q_bstride + (long)h * a.head_stride;
  const long kvh = a.kv_head_stride ? a.kv_head_stride : a.head_stride;
  const uint16_t* kbp = a.k + (long)b * a.k_bstride + (long)h * kvh;
  const uint16_t* vbp = a.v + (long)b * a.v_bstride + (long)h * kvh;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int kbeg = fa.kbegin ? fa.kbegin[b] : 0;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q = q0 + 16c + fr][dh = 32s + 8g .. +8]
  u16x8 qf[2][2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int q = min(q0 + 16 * c + fr, a.Tq - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[c][s] = *reinterpret_cast<const u16x8*>(qb + (long)q * a.q_ld + 32 * s + 8 * g);
  }
  f32x4 o[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < 2; ++c) o[i][c] = f32x4{0, 0, 0, 0};
  float mrow[2] = {-INFINITY, -INFINITY}, lrow[2] = {0.f, 0.f};
  const float sl2 = 0.125f * kLog2e;

  int kend = a.Tk;
  if (fa.causal) kend = min(a.Tk, (int)(blockIdx.x * 128 + 127 + fa.causal_off + 1));
  const int kstart = (kbeg / 64) * 64;
  for (int k0 = kstart; k0 < kend; k0 += 64) {
    // ---- stage K (swizzled) and V^T ----
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = tid + it * 256;
      const int key = i >> 3, piece = i & 7;
      u16x8 kv = u16x8{0, 0, 0, 0, 0, 0, 0, 0}, vv = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (k0 + key < a.Tk) {
        kv = *reinterpret_cast<const u16x8*>(kbp + (long)(k0 + key) * a.k_ld + piece * 8);
        vv = *reinterpret_cast<const u16x8*>(vbp + (long)(k0 + key) * a.v_ld + piece * 8);
      }
      *reinterpret_cast<u16x8*>(Ks + key * 64 + ((piece ^ (key & 7)) << 3)) = kv;
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(piece * 8 + e) * VTLD + key] = vv[e];
    }
    __syncthreads();
    // ---- S^T = K Q^T ----
    f32x4 st[4][2];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int key = kb * 16 + fr;
      u16x8 kf0 = *reinterpret_cast<const u16x8*>(Ks + key * 64 + (((0 * 4 + g) ^ (key & 7)) << 3));
      u16x8 kf1 = *reinterpret_cast<const u16x8*>(Ks + key * 64 + (((1 * 4 + g) ^ (key & 7)) << 3));
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f32x4 z = f32x4{0, 0, 0, 0};
        z = mfma16<T>(kf0, qf[c][0], z);
        st[kb][c] = mfma16<T>(kf1, qf[c][1], z);
      }
    }
    // ---- online softmax (query = 16c + fr on this lane; keys kb*16 + 4g + r) ----
    u16x8 pf[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int qi = q0 + 16 * c + fr;
      float tmax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + kb * 16 + 4 * g + r;
          bool ok = key < a.Tk && key >= kbeg;
          if (fa.causal) ok = ok && key <= qi + fa.causal_off;
          const float sv = ok ? st[kb][c][r] * sl2 : -INFINITY;
          st[kb][c][r] = sv;
          tmax = fmaxf(tmax, sv);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float mnew = fmaxf(mrow[c], tmax);
      const float msafe = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = exp2f(mrow[c] - msafe);
      mrow[c] = mnew;
      float psum = 0.f;
      float p[4][4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[kb][r] = exp2f(st[kb][c][r] - msafe);
          psum += p[kb][r];
        }
      lrow[c] = lrow[c] * alpha + psum;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db][c] *= alpha;
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        u16x8 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = from_f32<T>(p[2 * kc][r]);
          v[4 + r] = from_f32<T>(p[2 * kc + 1][r]);
        }
        pf[c][kc] = v;
      }
    }
    // ---- O^T += V^T P^T ----
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int dh = db * 16 + fr;
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        const u16x4 lo = *reinterpret_cast<const u16x4*>(Vt + dh * VTLD + kc * 32 + 4 * g);
        const u16x4 hi = *reinterpret_cast<const u16x4*>(Vt + dh * VTLD + kc * 32 + 16 + 4 * g);
        const u16x8 vf = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int c = 0; c < 2; ++c) o[db][c] = mfma16<T>(vf, pf[c][kc], o[db][c]);
      }
    }
    __syncthreads();
  }
  // ---- epilogue: lane holds O^T[dh = db*16 + 4g + r][q = 16c + fr] ----
  uint16_t* ob = a.o + (long)b * a.o_bstride + (long)h * a.head_stride;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float l = lrow[c];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    const int q = q0 + 16 * c + fr;
    if (q < a.Tq) {
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        u16x4 w;
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = from_f32<T>(o[db][c][r] * inv);
        *reinterpret_cast<u16x4*>(ob + (long)q * a.o_ld + db * 16 + 4 * g) = w;
      }
    }
  }
}

void launch_attn_flash(DT dt, const AttnArgs& a, int causal, int causal_off, const int* kbegin, hipStream_t st) {
  FlashArgs fa{a, causal, causal_off, kbegin};
  dim3 grid(cdiv(a.Tq, 128), a.H, a.B);
  if (dt == DT::BF16)
    hipLaunchKernelGGL(attn_flash_kernel<DT::BF16>, grid, dim3(256), 0, st, fa);
  else
    hipLaunchKernelGGL(attn_flash_kernel<DT::F16>, grid, dim3(256), 0, st, fa);
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Encoder self attention (non-causal, head_dim 64) on v_mfma_f32_32x32x16.  Workgroup = 4 waves x 32 queries
// of one (window, head); K/V tiles of 64 keys arrive by LDS-DMA (global_load_lds_dwordx4, double-buffered,
// the next tile in flight across the single barrier of each step).
//   S^T = K.Q^T: lane (c = l&31, h = l>>5) holds 16 scores of query c per 32-key block (keys
//     (r&3) + 8(r>>2) + 4h), so the row max is in-lane plus one permlane32_swap.
//   O^T += V^T.P^T takes the exponentiated scores straight from the accumulator registers as its B operand
//     (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"): no LDS round trip for P;
//     the V^T operand comes from the row-major V tile by ds_read_b64_tr_b16 (T10).
// Both LDS tiles are [64 keys][64 dims] with 16-B chunk c of row r stored at c ^ enc_sw(r) (swizzle applied on the
// DMA source address, the LDS image stays lane-linear).  enc_sw permutes bits 1..3 of the row so that both reads
// are bank-conflict-free under gfx950's lane grouping: the K ds_read_b128 (four 16-lane groups {0-3,12-15,20-27},
// ...: every group sees 16 distinct (row parity, chunk) slots) and the V ds_read_b64_tr_b16 (per 32-lane half,
// rows r and r + 2 of a 4-row block land in opposite chunk quads).  Plain c ^ (r & 7) measured 2.7 conflict
// cycles per LDS instruction (SQ_LDS_BANK_CONFLICT).
// ------------------------------------------------------------------------------------------------
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
template <DT T> __device__ inline f32x16 mfma32(const u16x8& a, const u16x8& b, f32x16 c);
template <> __device__ inline f32x16 mfma32<DT::BF16>(const u16x8& a, const u16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                 0);
}
template <> __device__ inline f32x16 mfma32<DT::F16>(const u16x8& a, const u16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// max of v over lanes l and l ^ 32: v_permlane32_swap exchanges the two 32-lane halves between its two
// operands, so of its two results one is this lane's value and the other the partner's, in either order
__device__ inline float max_pair32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(v, fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}

// eight f32 -> eight bf16 / f16 with the hardware round-to-nearest-even converts (v_cvt_pk_bf16_f32)
// (elements o .. o + 7 of a 16-float accumulator)
template <DT T> __device__ inline u16x8 pack8(const f32x16& v, int o);
template <> __device__ inline u16x8 pack8<DT::BF16>(const f32x16& v, int o) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[o + j];
  return __builtin_bit_cast(u16x8, r);
}
template <> __device__ inline u16x8 pack8<DT::F16>(const f32x16& v, int o) {
  f16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (_Float16)v[o + j];
  return __builtin_bit_cast(u16x8, r);
}

__device__ inline int enc_sw(int r) { return ((r >> 2) & 1) | (((r >> 3) & 1) << 1) | (((r >> 1) & 1) << 2); }

constexpr int kEncTile = 64;                       // keys per step
constexpr int kEncTileBytes = kEncTile * 64 * 2;   // one K or V tile
// NWV waves x 32 queries per workgroup share every K/V tile: the kernel is bound by the rate at which a CU fills
// its LDS from L2 (~11-13 B/clk/CU, MI355X_MICROARCH.md 'prologue HBM burst'; 4 waves: 10.6 B/clk measured), so
// the K/V bytes per query set its speed -- 8 waves halve them
template <DT T, int NWV, int MINW>
__global__ __launch_bounds__(64 * NWV, MINW) void enc_attn_kernel(AttnArgs a) {
  constexpr int QB = 32 * NWV, NP = 8 / NWV;  // queries per workgroup; K (and V) pieces each wave stages per tile
  // 1-D grid, XCD-grouped (§5.5 T1): the query tiles of one (window, head) run on one XCD, so its K/V stream is
  // fetched into that XCD's L2 once instead of once per tile
  const int nqt = (a.Tq + QB - 1) / QB, nwg = nqt * a.H * a.B;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  }
  const int qt = bid % nqt, bh = bid / nqt;
  const int h = bh % a.H, b = bh / a.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31, hl = lane >> 5;
  __shared__ __attribute__((aligned(16))) char lds[4 * kEncTileBytes];  // [buf][K | V]
  const uint16_t* qb = a.q + (long)b * a.q_bstride + (long)h * a.head_stride;
  const uint16_t* kb = a.k + (long)b * a.k_bstride + (long)h * a.head_stride;
  const uint16_t* vb = a.v + (long)b * a.v_bstride + (long)h * a.head_stride;
  const int q0 = qt * QB + wave * 32;
  const int Tk = a.Tk;
  const int ntiles = (Tk + kEncTile - 1) / kEncTile;

  // DMA staging: a tile is 8 pieces of 1 KiB (8 rows x 128 B); wave w stages K pieces w, w + NWV, .. and the same
  // V pieces.  Lane l covers row l >> 3 of its piece and reads source chunk (l & 7) ^ enc_sw(row).
  const int srow = lane >> 3;
  int schunk[NP];
  // per-lane source pointers of tile 0, advanced by a wave-uniform 64 rows per tile; only the last tile clamps
  const uint16_t* ksrc[NP];
  const uint16_t* vsrc[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int r = (wave + NWV * i) * 8 + srow;
    schunk[i] = ((lane & 7) ^ enc_sw(r)) * 8;
    ksrc[i] = kb + (long)r * a.k_ld + schunk[i];
    vsrc[i] = vb + (long)r * a.v_ld + schunk[i];
  }
  auto stage = [&](int t, int buf) {
    char* kd = lds + buf * 2 * kEncTileBytes;
    char* vd = kd + kEncTileBytes;
    const bool edge = (t + 1) * kEncTile > Tk;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int piece = wave + NWV * i;
      const uint16_t* ks = ksrc[i] + (long)t * kEncTile * a.k_ld;
      const uint16_t* vs = vsrc[i] + (long)t * kEncTile * a.v_ld;
      if (edge) {  // rows past Tk re-read row Tk - 1 (finite data; their scores are masked)
        const int key = min(t * kEncTile + piece * 8 + srow, Tk - 1);
        ks = kb + (long)key * a.k_ld + schunk[i];
        vs = vb + (long)key * a.v_ld + schunk[i];
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ks,
                                       (__attribute__((address_space(3))) void*)(kd + piece * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)vs,
                                       (__attribute__((address_space(3))) void*)(vd + piece * 1024), 16, 0, 0);
    }
  };
  stage(0, 0);

  // Q^T fragments (B operand): lane holds Q[q0 + c][16s + 8hl .. +8] for dim steps s = 0..3, pre-scaled by
  // C = log2(e) / sqrt(64) and rounded once to T, so the MFMA produces scores in log2 units directly (the
  // reference rounds its scaled q, and then its scores, to the same 16-bit type)
  const float C = 0.125f * kLog2e;
  u16x8 qf[4];
  {
    const int q = min(q0 + c, a.Tq - 1);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const u16x8 raw = *reinterpret_cast<const u16x8*>(qb + (long)q * a.q_ld + 16 * s2 + 8 * hl);
      f32x16 sc;
#pragma unroll
      for (int e = 0; e < 8; ++e) sc[e] = to_f32<T>(raw[e]) * C;
      qf[s2] = pack8<T>(sc, 0);
    }
  }
  f32x16 o[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  // m_run: this lane's query's softmax baseline (log2 units); negm = -m_run in every element is the QK^T
  // accumulator's initial value, so the scores come out of the MFMA already shifted (no per-score subtract)
  float m_run = 0.f, l_run = 0.f;
  f32x16 negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) negm[r] = 0.f;

  // per-lane LDS offsets.  K A-operand: row 32kb + c, chunk 2s + hl.
  const int krow_sw = enc_sw(c);  // rows 32 kb + c: bits 1..3 are c's
  // V^T A-operand by transposed reads: group G = lane >> 4 covers dims 16(G&1) .. +16 of keys base + 4(G>>1) + q;
  // lane 4q + p of the group addresses row (base + q), dims 16(G&1) + 4p .. +4
  const int G = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  int voff[2][2];  // [db][half]: rows 8 half + 4 (G >> 1) + tq of a 16-row group, dims 32 db + 16 (G & 1) + 4 tp
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = 8 * half + 4 * (G >> 1) + tq;
      const int col = 32 * db + 16 * (G & 1) + 4 * tp;
      voff[db][half] = row * 128 + (((col >> 3) ^ enc_sw(row)) << 4) + (col & 7) * 2;
    }
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t landed for every wave; every wave is done with buffer buf ^ 1
    if (t + 1 < ntiles) stage(t + 1, buf ^ 1);
    const char* Ks = lds + buf * 2 * kEncTileBytes;
    const char* Vs = Ks + kEncTileBytes;
    // ---- S^T = K.Q^T (two 32-key blocks) ----
    f32x16 st[2];
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
      const int row = 32 * kb2 + c;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const u16x8 kf = *reinterpret_cast<const u16x8*>(Ks + row * 128 + (((2 * s2 + hl) ^ krow_sw) << 4));
        st[kb2] = mfma32<T>(kf, qf[s2], s2 == 0 ? negm : st[kb2]);
      }
    }
    if ((t + 1) * kEncTile > Tk) {  // last, partial tile: keys past Tk never count
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t * kEncTile + 32 * kb2 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= Tk) st[kb2][r] = -INFINITY;
        }
    }
    // ---- online softmax on baseline-relative log2 scores ----
    float mx = st[0][0];
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[kb2][r]);
    mx = max_pair32(mx);
    // deferred rescale (cdna_hip_programming.md T13): the baseline moves only when this tile's max exceeds it by
    // more than 8, so P <= 2^8; the decision precedes this tile's exponentials, and O and l are rescaled together
    // with the same factor.  The first tile always moves the baseline to its max (alpha multiplies zeros).
    float ls = 0.f;
    if (__builtin_amdgcn_ballot_w64(mx > 8.0f || t == 0) != 0) {  // rare: wave-uniform branch
      const float d = (mx > 8.0f || t == 0) ? mx : 0.f;
      const float alpha = t == 0 ? 0.f : __builtin_amdgcn_exp2f(-d);  // t = 0: O and l are still zero
      m_run += d;
#pragma unroll
      for (int r = 0; r < 16; ++r) negm[r] = -m_run;
      l_run *= alpha;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
        for (int r = 0; r < 16; ++r) st[kb2][r] -= d;
    }
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(st[kb2][r]);
        st[kb2][r] = p;
        ls += p;
      }
    u16x8 pf[2][2];
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) pf[kb2][s2] = pack8<T>(st[kb2], 8 * s2);
    l_run += ls;
    // ---- O^T += V^T.P^T ----
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          u16x8 vf;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            // enc_sw only sees bits 1..3 of the row, so 32 kb + 16 s is a plain immediate offset
            const s16x4 v4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(Vs + voff[db][half] + (32 * kb2 + 16 * s2) * 128));
#pragma unroll
            for (int e = 0; e < 4; ++e) vf[4 * half + e] = (uint16_t)v4[e];
          }
          o[db] = mfma32<T>(vf, pf[kb2][s2], o[db]);
        }
      }
  }
  // ---- epilogue: lane holds O^T[dim 32db + (r&3) + 8(r>>2) + 4hl][query c] ----
  const float lt = l_run + __shfl_xor(l_run, 32);
  const float inv = lt > 0.f ? 1.0f / lt : 0.f;
  const int q = q0 + c;
  if (a.o8) {
    // MX-fp8 output (the A operand of the MX-fp8 out-projection): block db of this head's 64 dims is split over
    // lanes c and c + 32 (16 values each), which agree on its scale through one permlane32 swap
    if (q < a.Tq) {
      const long row = (long)b * a.Tq + q;
      uint8_t* ob = a.o8 + row * a.o8_ld + (long)h * 64;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        float am = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) am = fmaxf(am, fabsf(o[db][r] * inv));
        const int ex = mx8_exp(max_pair32(am));
        const float is = mx8_inv_scale(ex);
#pragma unroll
        for (int rg = 0; rg < 4; ++rg)
          *reinterpret_cast<uint32_t*>(ob + 32 * db + 8 * rg + 4 * hl) =
              mx8_pack4(o[db][4 * rg] * inv * is, o[db][4 * rg + 1] * inv * is, o[db][4 * rg + 2] * inv * is,
                        o[db][4 * rg + 3] * inv * is);
        if (hl == 0) a.os[row * a.os_ld + 2 * h + db] = (uint8_t)(ex + 127);
      }
    }
  } else if (q < a.Tq) {
    uint16_t* ob = a.o + (long)b * a.o_bstride + (long)h * a.head_stride + (long)q * a.o_ld;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = from_f32<T>(o[db][4 * rg + e] * inv);
        *reinterpret_cast<u16x4*>(ob + 32 * db + 8 * rg + 4 * hl) = w;
      }
  }
}

void launch_attn_encoder(DT dt, const AttnArgs& a, hipStream_t st) {
  if (!a.o8 && (a.head_stride % 8 != 0 || a.k_ld % 8 != 0 || a.v_ld % 8 != 0 || a.q_ld % 8 != 0 ||
                a.kv_head_stride != 0)) {
    launch_attn_flash(dt, a, 0, 0, nullptr, st);
    return;
  }
  // 8 waves at <= 128 VGPRs (two workgroups per CU); the 4-wave and the 256-VGPR forms measured no faster (round 5,
  // profiles/r05v_attn_form_ab/) and were removed
  const bool bf = dt == DT::BF16;
  dim3 grid(cdiv(a.Tq, 256) * a.H * a.B);
  if (bf) hipLaunchKernelGGL((enc_attn_kernel<DT::BF16, 8, 4>), grid, dim3(512), 0, st, a);
  else hipLaunchKernelGGL((enc_attn_kernel<DT::F16, 8, 4>), grid, dim3(512), 0, st, a);
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// decoder self attention for decode steps: workgroup = (head, row); the row's keys are its ancestry
// (anc[r][slot] = the cache row holding slot `slot` of row r's hypothesis; identity without beams).
// Thread = (key group kg = tid >> 3 of 32, 8-dim chunk c = tid & 7); per batch of 256 keys each thread
// holds 8 keys' K and V chunks in registers, all their loads issued before any arithmetic (ancestry ->
// K/V is the only dependent round trip).  Online softmax across batches; block-wide reductions via LDS.
// ------------------------------------------------------------------------------------------------
template <DT T>
__global__ __launch_bounds__(256) void dec_self_attn_kernel(DecAttnArgs a) {
  constexpr int J = 8;  // keys per thread per batch (32 key groups x 8 = 256 keys)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long probe_t0 = (a.tprobe && tid == 0) ? probe_clock() : 0ull;  // in-situ probe
  const int h = blockIdx.x;
  const int m = blockIdx.y;  // r * Tn + i
  const int r = m / a.Tn, i = m - r * a.Tn;
  const int slot_q = load_uniform_i32(a.slot0) + i;
  const int beg = a.pad ? load_uniform_i32(a.pad + r) : 0;
  const int kg = tid >> 3, c = tid & 7;
  const long kvR = a.kv_R;
  __shared__ float qs[64], kcur[64], vcur[64];
  __shared__ float red[2][4];
  __shared__ float fin[4][64];
  const int* anc = a.anc ? a.anc + (long)r * a.anc_ld : nullptr;

  // ---- this step's q / k / v of (row, head): from the QKV split-K partials or the stored q + cache slot ----
  if (a.qS > 0) {
    __shared__ float2 lnrow;
    const int part = tid >> 6, e = tid & 63;
    const int col = part * a.d + h * 64 + e;
    float p = 0.f;
    // the bias rides in the partials' load batch (the LN-fold branch below holds a barrier the compiler will not
    // hoist loads across)
    const float bcol = (tid < 192 && a.qbias && !a.ln_c1) ? a.qbias[col] : 0.f;
    if (tid < 192) {
      const float* src = a.qpart + (long)m * a.qpart_ld + col;
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = u < a.qS ? src[u * a.qpart_stride] : 0.f;  // qS <= 8: one batch
#pragma unroll
      for (int u = 0; u < 8; ++u) p += t[u];
    }
    if (a.ln_c1) {  // LN1 folded into the QKV weights: this row's statistics, merged by the fourth wave
      if (wave == 3) {
        const float2 st = row_ln_from_stats(a.ln_stats + (long)m * a.ln_ld, 1, a.d >> 4);
        if (lane == 0) lnrow = st;
      }
      __syncthreads();
    }
    if (tid < 192) {
      const float val = a.ln_c1 ? lnrow.y * (p - lnrow.x * a.ln_c1[col]) + a.ln_c2[col]
                                : p + bcol;
      const uint16_t hv = from_f32<T>(val);
      const float f = to_f32<T>(hv);
      if (part == 0) {
        qs[e] = f * 0.125f;
      } else {
        (part == 1 ? kcur : vcur)[e] = f;
        const_cast<uint16_t*>(part == 1 ? a.kc : a.vc)[((long)slot_q * kvR + r) * a.d + h * 64 + e] = hv;
      }
    }
  } else if (tid < 192) {
    const int part = tid >> 6, e = tid & 63;
    if (part == 0)
      qs[e] = to_f32<T>(a.q[(long)m * a.q_ld + h * 64 + e]) * 0.125f;
    else
      (part == 1 ? kcur : vcur)[e] = to_f32<T>((part == 1 ? a.kc : a.vc)[((long)slot_q * kvR + r) * a.d + h * 64 + e]);
  }

  float m_run = -INFINITY, l_run = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool first = true;
  for (int b0 = beg; b0 <= slot_q; b0 += 32 * J) {
    // ancestry, then every K / V load of the batch (keys < slot_q come from the cache)
    int row[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int key = b0 + kg + 32 * j;
      row[j] = (anc && key < slot_q) ? anc[key] : r;
    }
    u16x8 kv[J], vv[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int key = min(b0 + kg + 32 * j, slot_q);
      const long off = ((long)key * kvR + row[j]) * a.d + h * 64 + c * 8;
      kv[j] = *reinterpret_cast<const u16x8*>(a.kc + off);
      vv[j] = *reinterpret_cast<const u16x8*>(a.vc + off);
    }
    if (first) {
      __syncthreads();  // qs / kcur / vcur (and this step's cache slot) complete
      first = false;
    }
    float q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = qs[c * 8 + e];
    float sc[J];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int key = b0 + kg + 32 * j;
      float p = 0.f;
      if (key == slot_q) {
#pragma unroll
        for (int e = 0; e < 8; ++e) p += q[e] * kcur[c * 8 + e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) p += q[e] * to_f32<T>(kv[j][e]);
      }
      p = sum8_lanes(p);
      sc[j] = key <= slot_q ? p : -INFINITY;
      mx = fmaxf(mx, sc[j]);
    }
    mx = wave_max(mx);
    if (lane == 0) red[0][wave] = mx;
    __syncthreads();
    const float m_new = fmaxf(m_run, fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3])));
    __syncthreads();  // red reused by the next batch
    const float alpha = __expf(m_run - m_new);
    l_run *= alpha;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= alpha;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int key = b0 + kg + 32 * j;
      const float p = __expf(sc[j] - m_new);  // 0 for keys past slot_q
      if (c == 0) l_run += p;
      if (key == slot_q) {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += p * vcur[c * 8 + e];
      } else if (key < slot_q) {
        // (keys past slot_q re-read slot_q's cache entry, which this launch is still writing: whatever a previous
        // call left there -- NaN after a non-finite call -- must not meet their zero weights, 0 x NaN = NaN)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += p * to_f32<T>(vv[j][e]);
      }
    }
    m_run = m_new;
  }
  // reduce over the 8 key groups of the wave, then over the 4 waves
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    acc[e] += dpp_mov<kDppXor8>(acc[e]);
    acc[e] = sum_xor32(sum_xor16(acc[e]));
  }
  const float lw = wave_sum(l_run);
  if (lane == 0) red[1][wave] = lw;
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) fin[wave][c * 8 + e] = acc[e];
  }
  __syncthreads();
  if (tid < 64) {
    const float tot = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    const float o = (fin[0][tid] + fin[1][tid] + fin[2][tid] + fin[3][tid]) / tot;
    a.o[(long)m * a.d + h * 64 + tid] = from_f32<T>(o);
  }
  if (a.tprobe && tid == 0) probe_record(a.tprobe, *a.slot0, probe_t0);
}

void launch_self_attn(DT dt, const DecAttnArgs& a, hipStream_t st) {
  dim3 grid(a.H, a.R * a.Tn);
  if (dt == DT::BF16)
    hipLaunchKernelGGL(dec_self_attn_kernel<DT::BF16>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(dec_self_attn_kernel<DT::F16>, grid, dim3(256), 0, st, a);
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// decoder cross attention (decode step and prefill): workgroup = (head, window, key chunk x 16-query tile).
// The nq = rows_per_win * Tn query rows of a window share its K / V^T stream.
//
// Per wave, per 32-key block kb: S^T = K.Q^T on MFMA with the block's keys permuted so that lane (q = l&15,
// g = l>>4) ends up holding the scores of keys kb + 8g + 0..7 for query q -- exactly the A-operand layout of
// the following P.V MFMA (A = P[16 q][32 keys]).  B of P.V is V^T[dim][kb + 8g .. +8]: one 16-B
// load per lane from the transposed V image.  Softmax statistics are per lane (q = l&15) plus two xor
// shuffles across the four 16-lane groups; P goes to the MFMA as bf16/f16 hi + lo halves (two MFMAs), so
// the probabilities keep ~16 mantissa bits.  No LDS until the 4-wave combine at the end.
// KS > 1: each chunk writes a (max, sum, o[64]) record per query; the last arriving chunk merges them in order.
// ------------------------------------------------------------------------------------------------
constexpr int kMaxTk = kXS, kMaxSplits = 16;
#ifndef WMX_XATTN_OCC
#define WMX_XATTN_OCC 4  // waves per SIMD (4: best with two concurrent context groups, 3: best alone)
#endif
typedef __attribute__((address_space(1))) float gf32;

// chunk records [nwin][H][KS][nq][66]; one arrival counter per (window, head) in DecAttnArgs::xcnt
inline long cross_records_floats(int H, int nwin, int nq, int KS) { return (long)nwin * H * KS * nq * 66; }

// F8 (the fp8 decode of model dtype MX8): the K / V^T images are e4m3 (launch_crosskv_quant: one 16-byte lane piece
// = both dim halves of a key pair / two dim blocks of a key block, so half the wave loads of the 16-bit images),
// widened to the 16-bit MFMA operands in registers; the image scales enter exactly -- the K scale (a power of two)
// multiplies the queries before their 16-bit rounding, the V scale the merged output -- and with XQ the fused
// query projection's weights are 8-bit too (packed8_index, per-row scales a.wq_scale)
// FQ (with XQ): LN2 folded into the fused query projection (the mixed step); its own instantiation, so the default
// fused kernel does not carry the statistics registers (at the 128-VGPR cap of 4 waves per SIMD they spilled)
// (Round 5 measured and removed: window pairs per workgroup, an XCD remap of the heads, a barrier ordering the
// projection loads before the K loads, and the chunk records merged in the cross out-projection)
template <DT T, int KPW, int NWV, bool XQ = false, bool F8 = false, bool FQ = false>
__global__ __launch_bounds__(64 * NWV, KPW <= 2 ? WMX_XATTN_OCC : 1) void dec_cross_attn_kernel(DecAttnArgs a, int KS, int chunk, float* __restrict__ part) {
  constexpr int NT = 64 * NWV;
  const int h = blockIdx.x, w = blockIdx.y, zz = blockIdx.z;
  const int ks = zz % KS, qt = zz / KS;
  // wave index as a scalar: the K / V buffer loads below take their block offsets in the scalar soffset operand, and
  // a wave index the compiler cannot prove uniform turns every one of them into a readfirstlane waterfall loop
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int nq = a.rows_per_win * a.Tn;
  // in-situ probe: this workgroup's start / end, device wall-clock ticks
  const unsigned long long probe_t0 = (a.tprobe && tid == 0) ? probe_clock() : 0ull;
  auto probe_end = [&] {
    if (a.tprobe && tid == 0) probe_record(a.tprobe, *a.slot0, probe_t0);
  };
  const int i0 = qt * 16;  // first query (within the window) of this tile
  const int nqt = min(16, nq - i0);
  const int trows = nqt;  // the projection tile's rows: queries i0 .. i0 + nqt of window w
  const long row0 = (long)w * nq + i0;
  const int kc0 = ks * chunk, kc1 = min(a.Tk, kc0 + chunk);
  const int per = ((kc1 - kc0 + NWV - 1) / NWV + 31) / 32 * 32;  // keys per wave, whole 32-key blocks
  const int kw0 = kc0 + wave * per, kw1 = min(kc1, kw0 + per);
  constexpr int EB = F8 ? 1 : 2;  // image element bytes
  const char* kbase = reinterpret_cast<const char*>(a.ck) + ((long)w * a.x_wstride + (long)h * a.x_hstride) * EB;
  const char* vbase = reinterpret_cast<const char*>(a.cv) + ((long)w * a.x_wstride + (long)h * a.x_hstride) * EB;
  // fp8 images: their scales (scalar loads, issued first; read-only in this launch)
  float ksc = 1.f, vsc = 1.f;
  if constexpr (F8) {
    typedef const __attribute__((address_space(4))) float cf4;
    ksc = *(cf4*)(a.ck_scale + w * a.H + h);
    vsc = *(cf4*)(a.cv_scale + w * a.H + h);
  }

  // ---- first batch of K / V^T loads (issued before the q reduction so their latency overlaps it) ----
  // K A-fragment of block b, pair u, dim half hh: key kb + 8*(fr>>2) + 4u + (fr&3), dims 32hh + 8g .. +8
  // V^T B-fragment of block b, dim block db: V^T[16db + fr][kb + 8g .. +8]
  // (F8: kf[b][u][0] holds both dim halves' 16 bytes, vf[b][dp] the 16 bytes of dim blocks 2dp, 2dp + 1)
  u16x8 kf[KPW][2][2], vf[KPW][4];
  // buffer loads: one 32-bit lane offset per image, the block / half / dim-block offsets in the scalar operand;
  // keys past the image (kb + ... >= kXS) fall outside the descriptor's range and read as zeros
  const auto krs = __builtin_amdgcn_make_buffer_rsrc((void*)kbase, (short)0, kXS * 64 * EB, 0x00020000);
  const auto vrs = __builtin_amdgcn_make_buffer_rsrc((void*)vbase, (short)0, 64 * kXS * EB, 0x00020000);
  // fragment-major images (crossk_off / crossv_off): every load below is one contiguous 1 KiB wave piece
  const int loff = lane * 16;
  // 32-key block index kb0 / 32 + b (blocks past the image read as zeros)
  auto load_k = [&](int kb0) {
#pragma unroll
    for (int b = 0; b < KPW; ++b)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int hh = 0; hh < (F8 ? 1 : 2); ++hh)
          kf[b][u][hh] = __builtin_bit_cast(
              u16x8, __builtin_amdgcn_raw_buffer_load_b128(krs, loff, ((((kb0 >> 5) + b) * 2 + u) * (F8 ? 1 : 2) + hh) * 1024, WMX_KV_AUX));
  };
  auto load_v = [&](int kb0) {
#pragma unroll
    for (int b = 0; b < KPW; ++b)
#pragma unroll
      for (int db = 0; db < (F8 ? 2 : 4); ++db)
        vf[b][db] = __builtin_bit_cast(
            u16x8, __builtin_amdgcn_raw_buffer_load_b128(vrs, loff, (((kb0 >> 5) + b) * (F8 ? 2 : 4) + db) * 1024, WMX_KV_AUX));
  };
  auto load_batch = [&](int kb0) {
    load_k(kb0);
    load_v(kb0);
  };
  // per-wave fp32 tiles: the fused query projection's K-slice partials here, the softmax combine at the end
  __shared__ float so[NWV][16][65];
  __shared__ float2 qln[16];  // the tile's rows' LayerNorm (mean, rstd) of the folded query projection
  // ---- fused cross-q projection (a.wq): the wave's share of the K steps of the 16 x 64 tile q = qin . wq_h^T,
  //      one MFMA fragment per (k-step, 16-column block) from the packed layout (packed_w_elem / packed_a_elem);
  //      all of the wave's query-projection loads are issued BEFORE the first K / V batch, so its MFMAs wait only
  //      for them; rows past the tile repeat its last query (never stored) ----
  // (F8: a k-step is 64 deep, one 16-byte packed8 weight piece per column block and two A fragments)
  constexpr int QKU = F8 ? 3 : 5;
  const int qksteps = a.d >> (F8 ? 6 : 5);
  const int qkper = (qksteps + NWV - 1) / NWV;
  const int qk0 = wave * qkper, qk1 = min(qksteps, qk0 + qkper);
  u16x8 qav[QKU][F8 ? 2 : 1], qbv[QKU][4];
  constexpr bool fuse_q = XQ;  // (a.wq != null; the launcher picks the instantiation)
  // this thread's query column h 64 + (tid & 63) (the same for both of its elements below): its bias (and 8-bit
  // row scale) now, not after the projection's barrier
  const float qb_col = (fuse_q && a.qbias) ? a.qbias[h * 64 + (tid & 63)] : 0.f;
  const float qs_col = (fuse_q && F8) ? a.wq_scale[h * 64 + (tid & 63)] : 1.f;
  // LN2 folded into the query weights (the mixed step, dec_step_mixed): qin is the 16-bit residual x and
  // q = rstd_row (p - mean_row c1[col]) + c2[col]; the constants now, the row statistics right after the K batch
  constexpr bool fold_q = fuse_q && FQ;  // (launcher: FQ iff a.ln_c1 with a.wq)
  const float qc1_col = fold_q ? a.ln_c1[h * 64 + (tid & 63)] : 0.f;
  const float qc2_col = fold_q ? a.ln_c2[h * 64 + (tid & 63)] : 0.f;
  float2 lns[4];  // rows wave (lanes 0..31) and wave + 8 (lanes 32..63) of the tile: their statistics groups
  if (fuse_q) {
    const uint16_t* ap = a.qin + (row0 + min(fr, trows - 1)) * a.qin_ld + 8 * g;
    const uint16_t* wp = a.wq + (((long)h * 4 * qksteps) << 9) + lane * 8;  // (F8: the same 16-byte lane pieces)
#pragma unroll
    for (int u = 0; u < QKU; ++u) {
      // clamped into the matrix (also for a wave with no k-steps): finite duplicate data that meets a zeroed A
      // fragment below, never uninitialised registers (0 x NaN garbage would poison the tile)
      const int k = min(qk0 + u, qksteps - 1);
      if constexpr (F8) {
        qav[u][0] = *reinterpret_cast<const u16x8*>(ap + k * 64);
        qav[u][1] = *reinterpret_cast<const u16x8*>(ap + k * 64 + 32);
      } else {
        qav[u][0] = *reinterpret_cast<const u16x8*>(ap + k * 32);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) qbv[u][j] = stream_load(reinterpret_cast<const u16x8*>(wp + (((long)j * qksteps + k) << 9)));
    }
  }
  // K first (the query projection's MFMAs wait only for their own loads), V after them (needed after QK^T, softmax)
  // (fused path: unconditional -- a wave without keys reads past the image, zeros by the descriptor's range, and
  // never uses them; a conditional batch would make the compiler's waits for the projection's loads count as if
  // the K loads had not been issued, i.e. wait for them too)
  // (fold: the row statistics before the K batch, so the merge after the projection MFMAs waits for them and not
  // for the K batch)
  if (fold_q)  // rows wave and wave + 8 of the tile (clamped: rows past nqt are never used), merged after the MFMAs
    row_ln_stats_load2(a.ln_stats + ((long)w * nq + i0 + min(wave, nqt - 1)) * a.ln_ld,
                       a.ln_stats + ((long)w * nq + i0 + min(wave + 8, nqt - 1)) * a.ln_ld, a.d >> 4, lns);
  if (fuse_q)
    load_k(kw0);
  else if (kw0 < kw1)
    load_batch(kw0);
  __builtin_amdgcn_sched_barrier(0);  // keep the K batch in flight under the projection (the scheduler sinks it)
  if (fuse_q) {
    f32x4 qa[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) qa[j] = f32x4{0, 0, 0, 0};
    // branch-free: a k-step past the wave's share (clamped duplicate load) multiplies a zeroed A fragment, so no
    // MFMA is conditional and the compiler's waits stay counted per load
#pragma unroll
    for (int u = 0; u < QKU; ++u) {
      const u16x8 za = {0, 0, 0, 0, 0, 0, 0, 0};
      const u16x8 av = qk0 + u < qk1 ? qav[u][0] : za;
      if constexpr (F8) {
        const u16x8 av1 = qk0 + u < qk1 ? qav[u][F8 ? 1 : 0] : za;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          u16x8 blo, bhi;
          fp8x16_to16<T>(__builtin_bit_cast(u32x4, qbv[u][j]), blo, bhi);
          qa[j] = mfma16<T>(av, blo, qa[j]);
          qa[j] = mfma16<T>(av1, bhi, qa[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) qa[j] = mfma16<T>(av, qbv[u][j], qa[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) so[wave][4 * g + r][16 * j + fr] = qa[j][r];
    if (fold_q) {  // one row per half-wave; ordered before the q build by the barrier below
      const float2 st = row_ln_stats_merge2(lns, a.d >> 4);
      const int rq = wave + 8 * (lane >> 5);
      if ((lane & 31) == 0 && rq < nqt) qln[rq] = st;
    }
    load_v(kw0);
    __syncthreads();
  }

  // ---- the tile's queries into LDS (bf16/f16), one element per thread: q = bias + sum of the split-K partials in
  //      slice order, or the stored q; pre-scaled by log2(e) / sqrt(64) so the scores come out of the MFMA in
  //      log2 units (softmax on exp2, no per-score scaling) ----
  // (F8: times the K image's power-of-two scale, so S = K8 . q' = K . q exactly as with the dequantized image)
  const float kQScale = 0.125f * 1.4426950408889634f * ksc;
  __shared__ __attribute__((aligned(16))) uint16_t qsh[16][72];
  if (fold_q) {
    // (merged beside the projection, above)
  } else if (a.qS > 0 && a.ln_c1) {  // LN2 folded into the cross-q weights: the tile's row statistics, one wave per row
    for (int q = wave; q < nqt; q += NWV) {
      const float2 st = row_ln_from_stats(a.ln_stats + ((long)w * nq + i0 + q) * a.ln_ld, 1, a.d >> 4);
      if (lane == 0) qln[q] = st;
    }
    __syncthreads();
  }
  for (int t = tid; t < 16 * 64; t += NT) {
    const int q = t >> 6, e = t & 63;
    uint16_t v = 0;
    if (q < trows) {
      const long row = row0 + q;
      const int col = h * 64 + e;
      if (fuse_q) {  // the waves' K-slice partials in wave order, + bias
        float p = 0.f;
#pragma unroll
        for (int wv = 0; wv < NWV; ++wv) p += so[wv][q][e];
        v = from_f32<T>((fold_q ? qln[q].y * (p - qln[q].x * qc1_col) + qc2_col : p * qs_col + qb_col) * kQScale);
      } else if (a.qS > 0) {
        const float* src = a.qpart + row * a.qpart_ld + col;
        float tv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) tv[u] = u < a.qS ? src[u * a.qpart_stride] : 0.f;  // qS <= 8
        float p = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) p += tv[u];
        const float val = a.ln_c1 ? qln[q].y * (p - qln[q].x * a.ln_c1[col]) + a.ln_c2[col]
                                  : p + (a.qbias ? a.qbias[col] : 0.f);
        v = from_f32<T>(val * kQScale);
      } else {
        v = from_f32<T>(to_f32<T>(a.q[row * a.q_ld + col]) * kQScale);
      }
    }
    qsh[q][e] = v;
  }
  __syncthreads();
  // Q^T B-fragments: lane (col q = fr, g): dims 32hh + 8g .. +8
  const int qrow = fr;
  u16x8 qb[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) qb[hh] = *reinterpret_cast<const u16x8*>(&qsh[qrow][32 * hh + 8 * g]);

  // ---- online softmax over the wave's key range, P.V on MFMA ----
  float m_run = -INFINITY, l_run = 0.f;  // statistics of query fr (replicated over g)
  f32x4 o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = f32x4{0, 0, 0, 0};
  for (int kb0 = kw0; kb0 < kw1; kb0 += 32 * KPW) {
    if (kb0 != kw0) load_batch(kb0);  // (prefill only: decode chunks are one batch, loaded above)
    float sv[KPW][8];
    const bool whole = kb0 + 32 * KPW <= kw1;  // (wave-uniform) no key of the batch past the range: no masking
#pragma unroll
    for (int b = 0; b < KPW; ++b) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x4 acc = f32x4{0, 0, 0, 0};
        if constexpr (F8) {
          u16x8 k0, k1;
          fp8x16_to16<T>(__builtin_bit_cast(u32x4, kf[b][u][0]), k0, k1);
          acc = mfma16<T>(k0, qb[0], acc);
          acc = mfma16<T>(k1, qb[1], acc);
        } else {
          acc = mfma16<T>(kf[b][u][0], qb[0], acc);
          acc = mfma16<T>(kf[b][u][1], qb[1], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb0 + 32 * b + 8 * g + 4 * u + r;
          sv[b][4 * u + r] = (whole || key < kw1) ? acc[r] : -INFINITY;
        }
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int b = 0; b < KPW; ++b)
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, sv[b][j]);
    mx = max_xor32(max_xor16(mx));
    const float m_new = fmaxf(m_run, mx);
    float ls = 0.f;
#pragma unroll
    for (int b = 0; b < KPW; ++b)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = __builtin_amdgcn_exp2f(sv[b][j] - m_new);
        sv[b][j] = e;
        ls += e;
      }
    ls = sum_xor32(sum_xor16(ls));
    if (kb0 == kw0) {  // first batch: o and l are still zero (the only batch of a decode chunk)
      l_run = ls;
    } else {
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      l_run = l_run * alpha + ls;
      // o rows are queries 4g + r: their alpha lives in lane (4g + r) of any group
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ar = __shfl(alpha, 4 * g + r);
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db][r] *= ar;
      }
    }
    m_run = m_new;
#pragma unroll
    for (int b = 0; b < KPW; ++b) {
      u16x8 phi, plo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint16_t hi = from_f32<T>(sv[b][j]);
        phi[j] = hi;
        plo[j] = from_f32<T>(sv[b][j] - to_f32<T>(hi));
      }
      if constexpr (F8) {
#pragma unroll
        for (int dp = 0; dp < 2; ++dp) {
          u16x8 v0, v1;
          fp8x16_to16<T>(__builtin_bit_cast(u32x4, vf[b][dp]), v0, v1);
          o[2 * dp] = mfma16<T>(phi, v0, o[2 * dp]);
          o[2 * dp] = mfma16<T>(plo, v0, o[2 * dp]);
          o[2 * dp + 1] = mfma16<T>(phi, v1, o[2 * dp + 1]);
          o[2 * dp + 1] = mfma16<T>(plo, v1, o[2 * dp + 1]);
        }
      } else {
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          o[db] = mfma16<T>(phi, vf[b][db], o[db]);
          o[db] = mfma16<T>(plo, vf[b][db], o[db]);
        }
      }
    }
  }

  // ---- combine the NWV waves (LDS), then output or a chunk record ----
  __shared__ float sm[NWV][16], sl[NWV][16];
  if (g == 0) {
    sm[wave][fr] = m_run;
    sl[wave][fr] = l_run;
  }
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 4; ++r) so[wave][4 * g + r][16 * db + fr] = o[db][r];
  __syncthreads();
  for (int t = tid; t < nqt * 64; t += NT) {
    const int q = t >> 6, e = t & 63;
    float M = sm[0][q];
#pragma unroll
    for (int wv = 1; wv < NWV; ++wv) M = fmaxf(M, sm[wv][q]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int wv = 0; wv < NWV; ++wv) {
      const float f = sm[wv][q] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(sm[wv][q] - M);
      L += sl[wv][q] * f;
      O += so[wv][q][e] * f;
    }
    const long row = (long)w * nq + i0 + q;
    if (KS == 1) {
      a.o[row * a.d + h * 64 + e] = from_f32<T>(O / L * vsc);
    } else {
      // chunk record, stored write-through (sc1) so the last arriver can read it without an L2 release
      gf32* pr = (gf32*)(part + (((long)(w * a.H + h) * KS + ks) * nq + i0 + q) * 66);
      if (e == 0) {
        __hip_atomic_store(pr, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pr + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(pr + 2 + e, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (KS == 1) {
    probe_end();
    return;
  }
  // ---- in-launch merge (cdna_hip_programming.md Guideline 16, sc1 form): every storing wave drains its
  //      write-through stores, one lane takes a ticket; the workgroup drawing KS-1 merges the records in chunk
  //      order with sc1 loads (no acquire fence needed) and re-arms the counter for the next launch ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* cnt = a.xcnt;
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(cnt + w * a.H + h, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sm[0][0] = old == KS - 1 ? 1.f : 0.f;
  }
  __syncthreads();
  if (sm[0][0] == 0.f) {
    probe_end();
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // every record load is a buffer load with sc1 (aux 16): it bypasses this CU's L1, so no acquire is needed
  const float* wh = part + (long)(w * a.H + h) * KS * nq * 66;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)wh, (short)0, KS * nq * 66 * 4, 0x00020000);
  for (int t = tid; t < nq * 64; t += NT) {
    const int q = t >> 6, e = t & 63;
    float rec[kMaxSplits][3];
#pragma unroll
    for (int k = 0; k < kMaxSplits; ++k) {
      if (k < KS) {
        const int off = ((k * nq + q) * 66) * 4;
        rec[k][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 16));
        rec[k][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4, 0, 16));
        rec[k][2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + (2 + e) * 4, 0, 16));
      }
    }
    float M = -INFINITY;
#pragma unroll
    for (int k = 0; k < kMaxSplits; ++k)
      if (k < KS) M = fmaxf(M, rec[k][0]);
    float l = 0.f, o2 = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxSplits; ++k) {
      if (k < KS) {
        const float sc2 = rec[k][0] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(rec[k][0] - M);
        l = __builtin_fmaf(rec[k][1], sc2, l);
        o2 = __builtin_fmaf(rec[k][2], sc2, o2);
      }
    }
    a.o[((long)w * nq + q) * a.d + h * 64 + e] = from_f32<T>(o2 / l * vsc);
  }
  if (tid == 0) __hip_atomic_store(cnt + w * a.H + h, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  probe_end();
}

// key chunk per workgroup; WMX_CROSS_CHUNK overrides the default for tuning runs
static int cross_chunk(int Tk, int nq, bool f8) {
  static const int env = [] {
    const char* v = getenv("WMX_CROSS_CHUNK");
    return v ? atoi(v) : 0;
  }();
  if (nq > 16) return Tk;  // prefill: many query tiles already fill the chip
  if (env) return env;
  // large-v3, 2 groups x 4 windows, 8 waves per workgroup: 1024-key chunks (2 per window-head) 600-602 ms per call,
  // 768: 603-605, 512 with 4 waves: 610-625 (interleaved bench.py sweep, r01); 512 beat 256 with 4 waves;
  // unsplit (1504): 611-612 vs 591 (r01f).  fp8 images (half the bytes per key): 512-key chunks, 463 / 709x real
  // time at 8 / 16 windows against 1024's 457 / 645-659x, 768's 466 / 665x and unsplit's 442 / 704-707x
  // (profiles/r04_fp8_decode/, gpurun_out r04g / r04h)
  return f8 ? 512 : 1024;
}

size_t cross_attn_ws_floats(int H, int nwin, int nq_max) {
  return (size_t)cross_records_floats(H, nwin, nq_max, kMaxSplits);
}

template <DT T, bool F8>
static void launch_cross_t(const DecAttnArgs& a, float* ws, hipStream_t st) {
  const int nq = a.rows_per_win * a.Tn;
  const int nwin = a.R / a.rows_per_win;
  const int chunk = std::min(cross_chunk(a.Tk, nq, F8), a.Tk);
  const int KS = (a.Tk + chunk - 1) / chunk;
  const int QT = (nq + 15) / 16;
  WMX_CHECK(KS <= kMaxSplits, "cross attn: too many key chunks");
  WMX_CHECK(KS == 1 || chunk % 32 == 0, "cross attn: key chunks must be whole 32-key blocks");
  WMX_CHECK(KS == 1 || (ws != nullptr && a.xcnt != nullptr && nq <= 16), "cross attn: split workspace required");
  dim3 grid(a.H, nwin, KS * QT);
  // decode (nq <= 16): 8 waves per workgroup (a 1024-key chunk is one 128-key batch per wave); prefill: 4 waves
  // the fused query projection holds a wave's whole K share (<= 5 k-steps) in one load batch
  WMX_CHECK(!a.wq || (F8 ? (a.d / 64 + 7) / 8 <= 3 : (a.d / 32 + 7) / 8 <= 5),
            "cross attn: fused query projection: model width too large for one load batch per wave");
  WMX_CHECK(!a.wq || nq <= 16, "cross attn: the fused query projection runs on the 8-wave decode kernel");
  if (a.wq) {
    const int per_wave = ((chunk + 7) / 8 + 31) / 32;
    const bool fq = a.ln_c1 != nullptr;  // (16-bit only: launch_cross_attn's check)
#define WMX_XQ_LAUNCH(KPW)                                                                                           \
  if constexpr (!F8) {                                                                                             \
    if (fq) {                                                                                                      \
      hipLaunchKernelGGL((dec_cross_attn_kernel<T, KPW, 8, true, false, true>), grid, dim3(512), 0, st, a, KS, chunk, ws); \
      break;                                                                                                       \
    }                                                                                                              \
  }                                                                                                                \
  hipLaunchKernelGGL((dec_cross_attn_kernel<T, KPW, 8, true, F8>), grid, dim3(512), 0, st, a, KS, chunk, ws);
    switch (std::min(per_wave, 4)) {
      case 1: WMX_XQ_LAUNCH(1) break;
      case 2: WMX_XQ_LAUNCH(2) break;
      case 3: WMX_XQ_LAUNCH(3) break;
      default: WMX_XQ_LAUNCH(4) break;
    }
#undef WMX_XQ_LAUNCH
    return;
  }
  if (nq <= 16) {
    const int per_wave = ((chunk + 7) / 8 + 31) / 32;
    switch (std::min(per_wave, 4)) {
      case 1: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 1, 8, false, F8>), grid, dim3(512), 0, st, a, KS, chunk, ws); break;
      case 2: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 2, 8, false, F8>), grid, dim3(512), 0, st, a, KS, chunk, ws); break;
      case 3: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 3, 8, false, F8>), grid, dim3(512), 0, st, a, KS, chunk, ws); break;
      default: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 4, 8, false, F8>), grid, dim3(512), 0, st, a, KS, chunk, ws); break;
    }
    return;
  }
  const int per_wave = ((chunk + 3) / 4 + 31) / 32;  // 32-key blocks per wave
  switch (std::min(per_wave, 4)) {
    case 1: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 1, 4, false, F8>), grid, dim3(256), 0, st, a, KS, chunk, ws); break;
    case 2: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 2, 4, false, F8>), grid, dim3(256), 0, st, a, KS, chunk, ws); break;
    case 3: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 3, 4, false, F8>), grid, dim3(256), 0, st, a, KS, chunk, ws); break;
    default: hipLaunchKernelGGL((dec_cross_attn_kernel<T, 4, 4, false, F8>), grid, dim3(256), 0, st, a, KS, chunk, ws); break;
  }
}

void launch_cross_attn(DT dt, const DecAttnArgs& a, float* ws, hipStream_t st) {
  WMX_CHECK(a.Tk <= 1500 && a.d == a.H * 64, "cross attn: shape");
  WMX_CHECK(!a.wq || (a.qin && a.Tn == 1 && a.rows_per_win <= 16 && a.d % 32 == 0 && a.qin_ld >= a.d),
            "cross attn: fused query projection needs a decode step (one 16-query tile per window)");
  const bool f8 = a.ck_scale != nullptr;
  WMX_CHECK(!f8 || (a.cv_scale && (!a.wq || a.wq_scale)), "cross attn: fp8 images need their scales (and 8-bit query weights)");
  WMX_CHECK(f8 || !a.wq_scale, "cross attn: 8-bit query weights run with the fp8 images only");
  WMX_CHECK(!(a.wq && a.ln_c1) || (!a.wq_scale && a.ln_c2 && a.ln_stats && a.d / 16 <= 128 && a.ln_ld >= a.d / 16 && a.qS == 0),
            "cross attn: the LayerNorm-folded fused query projection is 16-bit only");
  if (dt == DT::BF16) {
    if (f8) launch_cross_t<DT::BF16, true>(a, ws, st);
    else launch_cross_t<DT::BF16, false>(a, ws, st);
  } else {
    if (f8) launch_cross_t<DT::F16, true>(a, ws, st);
    else launch_cross_t<DT::F16, false>(a, ws, st);
  }
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// raw cross-attention scores of the alignment heads: out[hh][m][s] = q_m . k_s / 8
// ------------------------------------------------------------------------------------------------
template <DT T, bool F8>
__global__ __launch_bounds__(256) void cross_scores_kernel(DecAttnArgs a, const int* heads, float* out) {
  const int hh = blockIdx.x, m = blockIdx.y;
  const int h = heads[hh];
  const int r = m / a.Tn;
  const int w = r / a.rows_per_win;
  __shared__ float qs[64];
  // (fp8 images: the K image's scale folded into the query, like the decode kernel)
  const float ksc = F8 ? a.ck_scale[w * a.H + h] : 1.f;
  if (threadIdx.x < 64) qs[threadIdx.x] = to_f32<T>(a.q[(long)m * a.q_ld + h * 64 + threadIdx.x]) * 0.125f * ksc;
  __syncthreads();
  const long ioff = (long)w * a.x_wstride + (long)h * a.x_hstride;
  for (int s = threadIdx.x; s < a.Tk; s += 256) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      u16x8 kv;
      if constexpr (F8) {
        const uint2 k8 = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(a.ck) + ioff + crossk8_off(s, c * 8));
        kv = fp8x8_to16<T>(k8.x, k8.y);
      } else {
        kv = *reinterpret_cast<const u16x8*>(a.ck + ioff + crossk_off(s, c * 8));
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += qs[c * 8 + e] * to_f32<T>(kv[e]);
    }
    out[((long)hh * gridDim.y + m) * a.Tk + s] = acc;
  }
}

void launch_cross_scores(DT dt, const DecAttnArgs& a, const int* heads, int nh, float* out, hipStream_t st) {
  dim3 grid(nh, a.R * a.Tn);
  const bool f8 = a.ck_scale != nullptr;
  if (dt == DT::BF16) {
    if (f8) hipLaunchKernelGGL((cross_scores_kernel<DT::BF16, true>), grid, dim3(256), 0, st, a, heads, out);
    else hipLaunchKernelGGL((cross_scores_kernel<DT::BF16, false>), grid, dim3(256), 0, st, a, heads, out);
  } else {
    if (f8) hipLaunchKernelGGL((cross_scores_kernel<DT::F16, true>), grid, dim3(256), 0, st, a, heads, out);
    else hipLaunchKernelGGL((cross_scores_kernel<DT::F16, false>), grid, dim3(256), 0, st, a, heads, out);
  }
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
