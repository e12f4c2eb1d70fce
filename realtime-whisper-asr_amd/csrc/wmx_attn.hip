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
__global__ __launch_bounds__(64) void dec_self_attn_kernel(DecAttnArgs a) {
  const int lane = threadIdx.x;
  const int h = blockIdx.x;
  const int m = blockIdx.y;  // r * Tn + i
  __shared__ float s[512];
  const int r = m / a.Tn, i = m - r * a.Tn;
  const int slot_q = *a.slot0 + i;
  const int beg = a.pad ? a.pad[r] : 0;
  const int gi = lane >> 3, j = lane & 7;
  float q[8];
  {
    const u16x8 qv = *reinterpret_cast<const u16x8*>(a.q + (long)m * a.q_ld + h * 64 + j * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = to_f32<T>(qv[e]) * 0.125f;
  }
  const int* anc = a.anc ? a.anc + (long)r * a.anc_ld : nullptr;
  float mx = -INFINITY;
  for (int s0 = beg; s0 <= slot_q; s0 += 8) {
    const int key = s0 + gi;
    float part = 0.f;
    if (key <= slot_q) {
      const int row = anc ? anc[key] : r;
      const u16x8 kv = *reinterpret_cast<const u16x8*>(a.kc + ((long)key * a.R + row) * a.d + h * 64 + j * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) part += q[e] * to_f32<T>(kv[e]);
    }
    part += __shfl_xor(part, 1);
    part += __shfl_xor(part, 2);
    part += __shfl_xor(part, 4);
    if (key <= slot_q) {
      if (j == 0) s[key - beg] = part;
      mx = fmaxf(mx, part);
    }
  }
  mx = wave_max(mx);
  __syncthreads();
  const int n = slot_q - beg + 1;
  float sum = 0.f;
  for (int t = lane; t < n; t += 64) {
    const float e = __expf(s[t] - mx);
    s[t] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int s0 = beg; s0 <= slot_q; s0 += 8) {
    const int key = s0 + gi;
    if (key <= slot_q) {
      const int row = anc ? anc[key] : r;
      const float p = s[key - beg];
      const u16x8 vv = *reinterpret_cast<const u16x8*>(a.vc + ((long)key * a.R + row) * a.d + h * 64 + j * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += p * to_f32<T>(vv[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    acc[e] += __shfl_xor(acc[e], 8);
    acc[e] += __shfl_xor(acc[e], 16);
    acc[e] += __shfl_xor(acc[e], 32);
  }
  if (gi == 0) {
    const float inv = 1.0f / sum;
    u16x8 ov;
#pragma unroll
    for (int e = 0; e < 8; ++e) ov[e] = from_f32<T>(acc[e] * inv);
    *reinterpret_cast<u16x8*>(a.o + (long)m * a.d + h * 64 + j * 8) = ov;
  }
}

void launch_self_attn(DT dt, const DecAttnArgs& a, hipStream_t st) {
  dim3 grid(a.H, a.R * a.Tn);
  if (dt == DT::BF16)
    hipLaunchKernelGGL(dec_self_attn_kernel<DT::BF16>, grid, dim3(64), 0, st, a);
  else
    hipLaunchKernelGGL(dec_self_attn_kernel<DT::F16>, grid, dim3(64), 0, st, a);
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// decoder cross attention for a decode step: one workgroup per (window, head); nq = rows_per_win*Tn <= 8
// ------------------------------------------------------------------------------------------------
constexpr int kMaxQ = 8, kMaxTk = 1536;

template <DT T>
__global__ __launch_bounds__(256) void dec_cross_attn_kernel(DecAttnArgs a) {
  const int h = blockIdx.x, w = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nq = a.rows_per_win * a.Tn;
  const int m0 = w * nq;  // rows of window w are contiguous: m = r*Tn + i, r in [w*rpw, (w+1)*rpw)
  __shared__ float sc[kMaxQ][kMaxTk];
  __shared__ float red[kMaxQ][4];
  __shared__ float fin[4][kMaxQ][64];
  // thread = (key group kg = tid >> 3 (32 groups), dh chunk c = tid & 7 (8 dims))
  const int kg = tid >> 3, c = tid & 7;
  float q[kMaxQ][8];
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi) {
    const int mq = m0 + min(qi, nq - 1);
    const u16x8 qv = *reinterpret_cast<const u16x8*>(a.q + (long)mq * a.q_ld + h * 64 + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[qi][e] = to_f32<T>(qv[e]) * 0.125f;
  }
  const uint16_t* kbase = a.ck + (long)w * a.Tk * a.ck_ld + h * 64;
  const uint16_t* vbase = kbase + a.d;
  float mx[kMaxQ];
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi) mx[qi] = -INFINITY;
  for (int s = kg; s < a.Tk; s += 32) {
    const u16x8 kv = *reinterpret_cast<const u16x8*>(kbase + (long)s * a.ck_ld + c * 8);
    float kf[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) kf[e] = to_f32<T>(kv[e]);
#pragma unroll
    for (int qi = 0; qi < kMaxQ; ++qi) {
      float p = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) p += q[qi][e] * kf[e];
      p += __shfl_xor(p, 1);
      p += __shfl_xor(p, 2);
      p += __shfl_xor(p, 4);
      mx[qi] = fmaxf(mx[qi], p);
      if (c == 0 && qi < nq) sc[qi][s] = p;
    }
  }
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi) {
    const float v = wave_max(mx[qi]);
    if (lane == 0) red[qi][wave] = v;
  }
  __syncthreads();
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi) mx[qi] = fmaxf(fmaxf(red[qi][0], red[qi][1]), fmaxf(red[qi][2], red[qi][3]));
  __syncthreads();
  float sum[kMaxQ];
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi) sum[qi] = 0.f;
  for (int s = tid; s < a.Tk; s += 256) {
#pragma unroll
    for (int qi = 0; qi < kMaxQ; ++qi) {
      if (qi < nq) {
        const float e = __expf(sc[qi][s] - mx[qi]);
        sc[qi][s] = e;
        sum[qi] += e;
      }
    }
  }
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi) {
    const float v = wave_sum(sum[qi]);
    if (lane == 0) red[qi][wave] = v;
  }
  __syncthreads();
  float acc[kMaxQ][8];
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[qi][e] = 0.f;
  for (int s = kg; s < a.Tk; s += 32) {
    const u16x8 vv = *reinterpret_cast<const u16x8*>(vbase + (long)s * a.ck_ld + c * 8);
    float vf[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) vf[e] = to_f32<T>(vv[e]);
#pragma unroll
    for (int qi = 0; qi < kMaxQ; ++qi) {
      if (qi < nq) {
        const float p = sc[qi][s];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[qi][e] += p * vf[e];
      }
    }
  }
  // reduce over the 8 key groups of a wave (lanes with equal c: xor 8, 16, 32), then over the 4 waves
#pragma unroll
  for (int qi = 0; qi < kMaxQ; ++qi)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = acc[qi][e];
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      acc[qi][e] = v;
    }
  if (lane < 8) {
#pragma unroll
    for (int qi = 0; qi < kMaxQ; ++qi)
#pragma unroll
      for (int e = 0; e < 8; ++e) fin[wave][qi][c * 8 + e] = acc[qi][e];
  }
  __syncthreads();
  for (int t = tid; t < nq * 64; t += 256) {
    const int qi = t >> 6, e = t & 63;
    const float tot = red[qi][0] + red[qi][1] + red[qi][2] + red[qi][3];
    const float v = (fin[0][qi][e] + fin[1][qi][e] + fin[2][qi][e] + fin[3][qi][e]) / tot;
    a.o[(long)(m0 + qi) * a.d + h * 64 + e] = from_f32<T>(v);
  }
}

void launch_cross_attn(DT dt, const DecAttnArgs& a, hipStream_t st) {
  const int nq = a.rows_per_win * a.Tn;
  WMX_CHECK(nq <= kMaxQ && a.Tk <= kMaxTk, "cross attn: too many queries per window");
  dim3 grid(a.H, a.R / a.rows_per_win);
  if (dt == DT::BF16)
    hipLaunchKernelGGL(dec_cross_attn_kernel<DT::BF16>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(dec_cross_attn_kernel<DT::F16>, grid, dim3(256), 0, st, a);
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
