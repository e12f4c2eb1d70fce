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
  const uint16_t* kbp = a.k + (long)b * a.k_bstride + (long)h * a.head_stride;
  const uint16_t* vbp = a.v + (long)b * a.v_bstride + (long)h * a.head_stride;
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

void launch_attn_encoder(DT dt, const AttnArgs& a, hipStream_t st) { launch_attn_flash(dt, a, 0, 0, nullptr, st); }

// ------------------------------------------------------------------------------------------------
// decoder self attention (decode step or small Tn), keys through the ancestry table
// ------------------------------------------------------------------------------------------------
template <DT T>
__global__ __launch_bounds__(256) void dec_self_attn_kernel(DecAttnArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.x;
  const int m = blockIdx.y;  // r * Tn + i
  __shared__ float s[512];
  __shared__ float red[4];
  __shared__ float fin[4][64];
  const int r = m / a.Tn, i = m - r * a.Tn;
  const int slot_q = *a.slot0 + i;
  const int beg = a.pad ? a.pad[r] : 0;
  const int gi = lane >> 3, j = lane & 7;  // 8 key groups x 8 dim chunks per wave
  float q[8];
  {
    const u16x8 qv = *reinterpret_cast<const u16x8*>(a.q + (long)m * a.q_ld + h * 64 + j * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = to_f32<T>(qv[e]) * 0.125f;
  }
  const int* anc = a.anc ? a.anc + (long)r * a.anc_ld : nullptr;
  constexpr int U = 4;  // per wave per iteration: 32 keys, 4 independent 16-B loads per lane
  float mx = -INFINITY;
  for (int s0 = beg + wave * 8 * U; s0 <= slot_q; s0 += 4 * 8 * U) {
    u16x8 kv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = min(s0 + 8 * u + gi, slot_q);
      const int row = anc ? anc[key] : r;
      kv[u] = *reinterpret_cast<const u16x8*>(a.kc + ((long)key * a.R + row) * a.d + h * 64 + j * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = s0 + 8 * u + gi;
      float part = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) part += q[e] * to_f32<T>(kv[u][e]);
      part += __shfl_xor(part, 1);
      part += __shfl_xor(part, 2);
      part += __shfl_xor(part, 4);
      if (key <= slot_q) {
        if (j == 0) s[key - beg] = part;
        mx = fmaxf(mx, part);
      }
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int n = slot_q - beg + 1;
  float sum = 0.f;
  for (int t = tid; t < n; t += 256) {
    const float e = __expf(s[t] - mx);
    s[t] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  if (lane == 0) red[wave] = sum;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int s0 = beg + wave * 8 * U; s0 <= slot_q; s0 += 4 * 8 * U) {
    u16x8 vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = min(s0 + 8 * u + gi, slot_q);
      const int row = anc ? anc[key] : r;
      vv[u] = *reinterpret_cast<const u16x8*>(a.vc + ((long)key * a.R + row) * a.d + h * 64 + j * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = s0 + 8 * u + gi;
      const float p = key <= slot_q ? s[key - beg] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += p * to_f32<T>(vv[u][e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    acc[e] += __shfl_xor(acc[e], 8);
    acc[e] += __shfl_xor(acc[e], 16);
    acc[e] += __shfl_xor(acc[e], 32);
  }
  if (gi == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) fin[wave][j * 8 + e] = acc[e];
  }
  __syncthreads();
  if (tid < 64) {
    const float tot = red[0] + red[1] + red[2] + red[3];
    const float o = (fin[0][tid] + fin[1][tid] + fin[2][tid] + fin[3][tid]) / tot;
    a.o[(long)m * a.d + h * 64 + tid] = from_f32<T>(o);
  }
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
// decoder cross attention for a decode step: one workgroup per (window, head); nq = rows_per_win*Tn <= 8
// ------------------------------------------------------------------------------------------------
constexpr int kMaxQ = 8, kMaxTk = 1536;
constexpr int kChunk = 384, kVPre = kChunk / 32;  // keys per workgroup, V rows prefetched per thread

// Q.K^T on MFMA: A = Q (16 query rows, nq valid) from registers, B = K^T straight from HBM (lane: key l&15,
// 16 B of head dims) — the dominant stream is read exactly once with 16-B loads, 8 key blocks in flight per
// wave.  Softmax in LDS, P.V on VALU (thread = 8 keys-apart group x 8 dims, 16-B V loads).  KS key splits per
// (window, head) keep all CUs streaming at small batch; partial (m, l, o) are merged by dec_cross_combine.
template <DT T>
__global__ __launch_bounds__(256) void dec_cross_attn_kernel(DecAttnArgs a, int KS, float* __restrict__ part,
                                                             int* __restrict__ cnt) {
  const int h = blockIdx.x, w = blockIdx.y, ks = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nq = a.rows_per_win * a.Tn;
  const int m0 = w * nq;
  const int chunk = ((a.Tk + KS - 1) / KS + 15) / 16 * 16;  // <= kChunk
  const int k0 = ks * chunk, k1 = min(a.Tk, k0 + chunk);
  const int nk = max(0, k1 - k0);
  __shared__ float sc[kMaxQ][kChunk + 4];
  __shared__ float red[kMaxQ][4];
  __shared__ float fin[4][kMaxQ][64];
  const uint16_t* kbase = a.ck + (long)w * a.Tk * a.ck_ld + h * 64;
  const uint16_t* vbase = kbase + a.d;
  // P.V mapping: thread = (key group kg = tid >> 3 of 32, dims c*8 .. c*8+7); prefetch all its V rows now
  const int kg = tid >> 3, c = tid & 7;
  u16x8 vpre[kVPre];
#pragma unroll
  for (int i = 0; i < kVPre; ++i) {
    const int t = min(kg + 32 * i, nk - 1);
    vpre[i] = *reinterpret_cast<const u16x8*>(vbase + (long)(k0 + max(t, 0)) * a.ck_ld + c * 8);
  }
  // Q fragments: lane row q = lane & 15, dims 32s + 8(lane>>4) .. +8
  const int fr = lane & 15, g = lane >> 4;
  u16x8 qa[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    u16x8 z = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (fr < nq) z = *reinterpret_cast<const u16x8*>(a.q + (long)(m0 + fr) * a.q_ld + h * 64 + 32 * s2 + 8 * g);
    qa[s2] = z;
  }
  // ---- scores: wave handles key blocks wave, wave+4, ... (<= 6 per wave), all loads issued first ----
  const int nblk = (nk + 15) / 16;
  constexpr int NB = kChunk / 16 / 4;  // 6
  u16x8 kb[NB][2];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int key = min(k0 + (wave + 4 * u) * 16 + fr, a.Tk - 1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) kb[u][s2] = *reinterpret_cast<const u16x8*>(kbase + (long)key * a.ck_ld + 32 * s2 + 8 * g);
  }
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int blk = wave + 4 * u;
    if (blk >= nblk) break;
    f32x4 acc = f32x4{0, 0, 0, 0};
    acc = mfma16<T>(qa[0], kb[u][0], acc);
    acc = mfma16<T>(qa[1], kb[u][1], acc);
    const int kl = blk * 16 + fr;  // lane holds S[q = 4g + r][key kl]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 4 * g + r;
      if (q < nq && kl < nk) sc[q][kl] = acc[r] * 0.125f;
    }
  }
  __syncthreads();
  // ---- softmax (partial over this key range) ----
  float mx[kMaxQ];
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) {
    float v = -INFINITY;
    if (q < nq)
      for (int t = tid; t < nk; t += 256) v = fmaxf(v, sc[q][t]);
    v = wave_max(v);
    if (lane == 0) red[q][wave] = v;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) mx[q] = fmaxf(fmaxf(red[q][0], red[q][1]), fmaxf(red[q][2], red[q][3]));
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) {
    float sum = 0.f;
    if (q < nq)
      for (int t = tid; t < nk; t += 256) {
        const float e = __expf(sc[q][t] - mx[q]);
        sc[q][t] = e;
        sum += e;
      }
    sum = wave_sum(sum);
    if (lane == 0) red[q][wave] = sum;
  }
  __syncthreads();
  // ---- P.V from the prefetched V rows ----
  float acc[kMaxQ][8];
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[q][e] = 0.f;
#pragma unroll
  for (int i = 0; i < kVPre; ++i) {
    const int t = kg + 32 * i;
    if (t < nk) {
      float vf[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) vf[e] = to_f32<T>(vpre[i][e]);
#pragma unroll
      for (int q = 0; q < kMaxQ; ++q) {
        if (q < nq) {
          const float p = sc[q][t];
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[q][e] += p * vf[e];
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) {
    if (q < nq) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = acc[q][e];
        v += __shfl_xor(v, 8);
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        acc[q][e] = v;
      }
    }
  }
  if (lane < 8) {
#pragma unroll
    for (int q = 0; q < kMaxQ; ++q)
      if (q < nq)
#pragma unroll
        for (int e = 0; e < 8; ++e) fin[wave][q][c * 8 + e] = acc[q][e];
  }
  __syncthreads();
  for (int t = tid; t < nq * 64; t += 256) {
    const int q = t >> 6, e = t & 63;
    const float tot = red[q][0] + red[q][1] + red[q][2] + red[q][3];
    const float o = fin[0][q][e] + fin[1][q][e] + fin[2][q][e] + fin[3][q][e];
    if (KS == 1) {
      a.o[(long)(m0 + q) * a.d + h * 64 + e] = from_f32<T>(o / tot);
    } else {
      // partial record per (window, head, split, q): [m, l, o[64]]
      float* pr = part + ((((long)w * a.H + h) * KS + ks) * kMaxQ + q) * 66;
      if (e == 0) {
        pr[0] = mx[q];
        pr[1] = tot;
      }
      pr[2 + e] = o;
    }
  }
  if (KS == 1) return;
  // ---- the last of the KS workgroups of (window, head) merges the partials (cdna_hip_programming.md
  //      Guideline 16: drained plain stores -> agent release -> counter; last arriver: agent acquire -> loads) ----
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(cnt + w * a.H + h, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == KS - 1;
  }
  __syncthreads();
  if (!last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int t = tid; t < nq * 64; t += 256) {
    const int q = t >> 6, e = t & 63;
    const float* pr = part + (((long)w * a.H + h) * KS * kMaxQ + q) * 66;
    float M = -INFINITY;
    for (int k = 0; k < KS; ++k) M = fmaxf(M, pr[(long)k * kMaxQ * 66]);
    float l = 0.f, o = 0.f;
    for (int k = 0; k < KS; ++k) {
      const float* x = pr + (long)k * kMaxQ * 66;
      const float sc2 = __expf(x[0] - M);
      l += x[1] * sc2;
      o += x[2 + e] * sc2;
    }
    a.o[(long)(m0 + q) * a.d + h * 64 + e] = from_f32<T>(o / l);
  }
  if (tid == 0) __hip_atomic_store(cnt + w * a.H + h, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int cross_attn_splits(int Tk) { return (Tk + kChunk - 1) / kChunk; }

// partial records + one arrival counter per (window, head) (the counters must start at 0; the last arriver resets)
size_t cross_attn_ws_floats(int H, int nwin) { return (size_t)nwin * H * 8 * kMaxQ * 66 + (size_t)nwin * H; }

void launch_cross_attn(DT dt, const DecAttnArgs& a, float* ws, hipStream_t st) {
  const int nq = a.rows_per_win * a.Tn;
  WMX_CHECK(nq <= kMaxQ && a.Tk <= kMaxTk, "cross attn: too many queries per window");
  const int nwin = a.R / a.rows_per_win;
  const int KS = cross_attn_splits(a.Tk);
  WMX_CHECK(KS == 1 || ws != nullptr, "cross attn: split workspace required");
  dim3 grid(a.H, nwin, KS);
  int* cnt = ws ? reinterpret_cast<int*>(ws + (size_t)nwin * a.H * 8 * kMaxQ * 66) : nullptr;
  if (dt == DT::BF16)
    hipLaunchKernelGGL(dec_cross_attn_kernel<DT::BF16>, grid, dim3(256), 0, st, a, KS, ws, cnt);
  else
    hipLaunchKernelGGL(dec_cross_attn_kernel<DT::F16>, grid, dim3(256), 0, st, a, KS, ws, cnt);
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// raw cross-attention scores of the alignment heads: out[hh][m][s] = q_m . k_s / 8
// ------------------------------------------------------------------------------------------------
template <DT T>
__global__ __launch_bounds__(256) void cross_scores_kernel(DecAttnArgs a, const int* heads, float* out) {
  const int hh = blockIdx.x, m = blockIdx.y;
  const int h = heads[hh];
  const int r = m / a.Tn;
  const int w = r / a.rows_per_win;
  __shared__ float qs[64];
  if (threadIdx.x < 64) qs[threadIdx.x] = to_f32<T>(a.q[(long)m * a.q_ld + h * 64 + threadIdx.x]) * 0.125f;
  __syncthreads();
  const uint16_t* kbase = a.ck + (long)w * a.Tk * a.ck_ld + h * 64;
  for (int s = threadIdx.x; s < a.Tk; s += 256) {
    const uint16_t* kp = kbase + (long)s * a.ck_ld;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const u16x8 kv = *reinterpret_cast<const u16x8*>(kp + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += qs[c * 8 + e] * to_f32<T>(kv[e]);
    }
    out[((long)hh * gridDim.y + m) * a.Tk + s] = acc;
  }
}

void launch_cross_scores(DT dt, const DecAttnArgs& a, const int* heads, int nh, float* out, hipStream_t st) {
  dim3 grid(nh, a.R * a.Tn);
  if (dt == DT::BF16)
    hipLaunchKernelGGL(cross_scores_kernel<DT::BF16>, grid, dim3(256), 0, st, a, heads, out);
  else
    hipLaunchKernelGGL(cross_scores_kernel<DT::F16>, grid, dim3(256), 0, st, a, heads, out);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
