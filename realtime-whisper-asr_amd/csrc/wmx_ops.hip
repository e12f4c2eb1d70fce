// Memory-bound helper kernels: LayerNorm (fp32 residual -> 16-bit GEMM operand), conv im2col, token+position
// embedding, dtype conversion, and the build-owned synthetic weight generator (same counter PRNG as
// oracle/whisper_np.py prng_uniform, bit-exact).
#include <cstdlib>

#include "wmx_common.h"
#include "wmx_kernels.h"

namespace wmx {

// ---------------- LayerNorm: one wave per row, two-pass (mean, then centred variance), eps 1e-5 ----------------
// A wave's share of a row is float4 columns lane + 64 i, i < (n4 + 63) / 64 <= 8.  The trip count is uniform and
// the addresses are clamped into the row, so every load of the row (and of gamma / beta) is issued in one batch
// before any use: with per-lane `c < n4` guards the compiler closed each guarded load with a vmcnt(0) wait, one
// round trip per float4 (16 per row).  Lanes past the row (c >= n4, d % 256 != 0) drop out through selects.
__device__ __forceinline__ void row_load8(const float4* __restrict__ p, int n4, int lane, float4 (&v)[8]) {
  const int nit = (n4 + 63) >> 6;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < nit) v[i] = p[min(lane + i * 64, n4 - 1)];
}

// the encoder fold's residual rows are two 16-bit planes, x = hi + lo (wmx_gemm.hip epi_rows64_lns): XLO != nullptr
// reads them instead of an fp32 row
template <DT T>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, const int* __restrict__ rows_idx,
                                                        const float* __restrict__ g, const float* __restrict__ bb,
                                                        uint16_t* __restrict__ out, int rows, int d,
                                                        const uint16_t* __restrict__ xlo) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int src = rows_idx ? rows_idx[row] : row;
  const int n4 = d >> 2, nit = (n4 + 63) >> 6;  // d <= 2048
  float4 v[8], gg[8], be[8];
  if (xlo) {
    const u16x4* ph = reinterpret_cast<const u16x4*>(reinterpret_cast<const uint16_t*>(x) + (long)src * d);
    const u16x4* pl = reinterpret_cast<const u16x4*>(xlo + (long)src * d);
    u16x4 h[8], l[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < nit) {
        h[i] = ph[min(lane + i * 64, n4 - 1)];
        l[i] = pl[min(lane + i * 64, n4 - 1)];
      }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < nit)
        v[i] = make_float4(to_f32<T>(h[i][0]) + to_f32<T>(l[i][0]), to_f32<T>(h[i][1]) + to_f32<T>(l[i][1]),
                           to_f32<T>(h[i][2]) + to_f32<T>(l[i][2]), to_f32<T>(h[i][3]) + to_f32<T>(l[i][3]));
  } else {
    row_load8(reinterpret_cast<const float4*>(x + (long)src * d), n4, lane, v);
  }
  row_load8(reinterpret_cast<const float4*>(g), n4, lane, gg);
  row_load8(reinterpret_cast<const float4*>(bb), n4, lane, be);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < nit) s += lane + i * 64 < n4 ? (v[i].x + v[i].y) + (v[i].z + v[i].w) : 0.f;
  const float mean = wave_sum(s) / d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < nit) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, e = v[i].w - mean;
      q += lane + i * 64 < n4 ? a * a + b * b + cc * cc + e * e : 0.f;
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / d + 1e-5f);
  uint16_t* o = out + (long)row * d;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + i * 64;
    if (i < nit && c < n4) {
      u16x4 w;
      w[0] = from_f32<T>((v[i].x - mean) * rstd * gg[i].x + be[i].x);
      w[1] = from_f32<T>((v[i].y - mean) * rstd * gg[i].y + be[i].y);
      w[2] = from_f32<T>((v[i].z - mean) * rstd * gg[i].z + be[i].z);
      w[3] = from_f32<T>((v[i].w - mean) * rstd * gg[i].w + be[i].w);
      reinterpret_cast<u16x4*>(o)[c] = w;
    }
  }
}

void launch_layernorm_rows(DT dt, const float* x, const int* rows_idx, const float* g, const float* b, uint16_t* out,
                           int rows, int d, hipStream_t st) {
  if (rows <= 0) return;
  WMX_CHECK(d % 4 == 0 && d <= 2048, "layernorm: d");
  dim3 grid(cdiv(rows, 4));
  if (dt == DT::BF16)
    hipLaunchKernelGGL(layernorm_kernel<DT::BF16>, grid, dim3(256), 0, st, x, rows_idx, g, b, out, rows, d, nullptr);
  else
    hipLaunchKernelGGL(layernorm_kernel<DT::F16>, grid, dim3(256), 0, st, x, rows_idx, g, b, out, rows, d, nullptr);
  WMX_HIP(hipGetLastError());
}

void launch_layernorm_split(DT dt, const uint16_t* xhi, const uint16_t* xlo, const float* g, const float* b,
                            uint16_t* out, int rows, int d, hipStream_t st) {
  if (rows <= 0) return;
  WMX_CHECK(d % 4 == 0 && d <= 2048, "layernorm: d");
  const float* x = reinterpret_cast<const float*>(xhi);
  dim3 grid(cdiv(rows, 4));
  if (dt == DT::BF16)
    hipLaunchKernelGGL(layernorm_kernel<DT::BF16>, grid, dim3(256), 0, st, x, nullptr, g, b, out, rows, d, xlo);
  else
    hipLaunchKernelGGL(layernorm_kernel<DT::F16>, grid, dim3(256), 0, st, x, nullptr, g, b, out, rows, d, xlo);
  WMX_HIP(hipGetLastError());
}

void launch_layernorm(DT dt, const float* x, const float* g, const float* b, uint16_t* out, int rows, int d,
                      hipStream_t st) {
  launch_layernorm_rows(dt, x, nullptr, g, b, out, rows, d, st);
}

// ---------------- LayerNorm straight to MX-fp8 (encoder, MX-fp8 mode): the same two-pass statistics as
// layernorm_kernel; the 8 lanes holding a 32-column block (4 columns each) agree on its e8m0 scale ----------------
__global__ __launch_bounds__(256) void layernorm_mx8_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                            const float* __restrict__ bb, uint8_t* __restrict__ q,
                                                            uint8_t* __restrict__ sc, int rows, int d) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int n4 = d >> 2, nit = (n4 + 63) >> 6;  // d <= 2048
  float4 v[8], gg[8], be[8];  // one load batch (row_load8)
  row_load8(reinterpret_cast<const float4*>(x + (long)row * d), n4, lane, v);
  row_load8(reinterpret_cast<const float4*>(g), n4, lane, gg);
  row_load8(reinterpret_cast<const float4*>(bb), n4, lane, be);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < nit) s += lane + i * 64 < n4 ? (v[i].x + v[i].y) + (v[i].z + v[i].w) : 0.f;
  const float mean = wave_sum(s) / d;
  float qq = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < nit) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, e = v[i].w - mean;
      qq += lane + i * 64 < n4 ? a * a + b * b + cc * cc + e * e : 0.f;
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(qq) / d + 1e-5f);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + i * 64;
    if (i < nit && c < n4) {  // n4 is a multiple of 8 (d % 32 == 0): a block's 8 lanes are all inside or all outside
      const float y0 = (v[i].x - mean) * rstd * gg[i].x + be[i].x, y1 = (v[i].y - mean) * rstd * gg[i].y + be[i].y;
      const float y2 = (v[i].z - mean) * rstd * gg[i].z + be[i].z, y3 = (v[i].w - mean) * rstd * gg[i].w + be[i].w;
      const int ex = mx8_exp(max8_lanes(fmaxf(fmaxf(fabsf(y0), fabsf(y1)), fmaxf(fabsf(y2), fabsf(y3)))));
      const float is = mx8_inv_scale(ex);
      reinterpret_cast<uint32_t*>(q + (long)row * d)[c] = mx8_pack4(y0 * is, y1 * is, y2 * is, y3 * is);
      if ((lane & 7) == 0) sc[(long)row * (d >> 5) + (c >> 3)] = (uint8_t)(ex + 127);
    }
  }
}

// the same for d == 256 * NIT (d 1024, 1280): unguarded loads, and the gain / bias vectors read in the store loop
// (L2-resident) instead of held beside the row (46 VGPRs at R = 1 against the generic kernel's 110).  A wave takes R
// rows with all their loads in one batch: at R = 2 the 12000 rows of 8 large-v3 windows are 6000 waves, which fit the
// chip's wave slots in one round instead of 1.5
#ifndef WMX_LNMX_T
#define WMX_LNMX_T 1
#endif
#ifndef WMX_LNMX_R
#define WMX_LNMX_R 1
#endif
template <int NIT, int R>
__global__ __launch_bounds__(256) void layernorm_mx8_exact_kernel(const float* __restrict__ x,
                                                                  const float* __restrict__ g,
                                                                  const float* __restrict__ bb, uint8_t* __restrict__ q,
                                                                  uint8_t* __restrict__ sc, int rows) {
  constexpr int d = 256 * NIT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + wave) * R;
  if (row0 >= rows) return;
  float4 v[R][NIT];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const float4* xr = reinterpret_cast<const float4*>(x + (long)min(row0 + j, rows - 1) * d);
#pragma unroll
    for (int i = 0; i < NIT; ++i) v[j][i] = xr[lane + i * 64];
  }
  float mean[R], rstd[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NIT; ++i) s += (v[j][i].x + v[j][i].y) + (v[j][i].z + v[j][i].w);
    mean[j] = wave_sum(s) / d;
  }
#pragma unroll
  for (int j = 0; j < R; ++j) {
    float qq = 0.f;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const float a = v[j][i].x - mean[j], b = v[j][i].y - mean[j], cc = v[j][i].z - mean[j], e = v[j][i].w - mean[j];
      qq += a * a + b * b + cc * cc + e * e;
    }
    rstd[j] = 1.0f / sqrtf(wave_sum(qq) / d + 1e-5f);
  }
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int c = lane + i * 64;
    const float4 gg = reinterpret_cast<const float4*>(g)[c], be = reinterpret_cast<const float4*>(bb)[c];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (row0 + j >= rows) break;
      const float m = mean[j], r = rstd[j];
      const float y0 = (v[j][i].x - m) * r * gg.x + be.x, y1 = (v[j][i].y - m) * r * gg.y + be.y;
      const float y2 = (v[j][i].z - m) * r * gg.z + be.z, y3 = (v[j][i].w - m) * r * gg.w + be.w;
      const int ex = mx8_exp(max8_lanes(fmaxf(fmaxf(fabsf(y0), fabsf(y1)), fmaxf(fabsf(y2), fabsf(y3)))));
      const float is = mx8_inv_scale(ex);
      reinterpret_cast<uint32_t*>(q + (long)(row0 + j) * d)[c] = mx8_pack4(y0 * is, y1 * is, y2 * is, y3 * is);
      if ((lane & 7) == 0) sc[(long)(row0 + j) * (d >> 5) + (c >> 3)] = (uint8_t)(ex + 127);
    }
  }
}

void launch_layernorm_mx8(const float* x, const float* g, const float* b, uint8_t* q, uint8_t* s, int rows, int d,
                          hipStream_t st) {
  if (rows <= 0) return;
  WMX_CHECK(d % 32 == 0 && d <= 2048, "layernorm_mx8: d");
  constexpr int R = WMX_LNMX_R;
  if (WMX_LNMX_T && d == 1280)
    hipLaunchKernelGGL((layernorm_mx8_exact_kernel<5, R>), dim3(cdiv(rows, 4 * R)), dim3(256), 0, st, x, g, b, q, s,
                       rows);
  else if (WMX_LNMX_T && d == 1024)
    hipLaunchKernelGGL((layernorm_mx8_exact_kernel<4, R>), dim3(cdiv(rows, 4 * R)), dim3(256), 0, st, x, g, b, q, s,
                       rows);
  else
    hipLaunchKernelGGL(layernorm_mx8_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, g, b, q, s, rows, d);
  WMX_HIP(hipGetLastError());
}

// ---------------- 16-bit rows -> MX-fp8 (weight preparation): one thread per 32-element block ----------------
template <DT T>
__global__ __launch_bounds__(256) void mx8_quantize_rows_kernel(const uint16_t* __restrict__ src, long rows, int K,
                                                                uint8_t* __restrict__ q, uint8_t* __restrict__ sc) {
  const int nb = K >> 5;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * nb) return;
  const long row = i / nb;
  const int b = (int)(i - row * nb);
  const uint16_t* p = src + row * K + 32 * b;
  float v[32];
  float am = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const u16x8 h = *reinterpret_cast<const u16x8*>(p + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[8 * c + e] = to_f32<T>(h[e]);
      am = fmaxf(am, fabsf(v[8 * c + e]));
    }
  }
  const int ex = mx8_exp(am);
  const float is = mx8_inv_scale(ex);
  uint32_t* o = reinterpret_cast<uint32_t*>(q + row * K + 32 * b);
#pragma unroll
  for (int w = 0; w < 8; ++w) o[w] = mx8_pack4(v[4 * w] * is, v[4 * w + 1] * is, v[4 * w + 2] * is, v[4 * w + 3] * is);
  sc[row * nb + b] = (uint8_t)(ex + 127);
}

void launch_mx8_quantize_rows(DT dt, const uint16_t* src, long rows, int K, uint8_t* q, uint8_t* s, hipStream_t st) {
  WMX_CHECK(K % 32 == 0, "mx8 quantize: K");
  const long n = rows * (K / 32);
  if (n <= 0) return;
  if (dt == DT::BF16)
    hipLaunchKernelGGL(mx8_quantize_rows_kernel<DT::BF16>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, rows, K, q, s);
  else
    hipLaunchKernelGGL(mx8_quantize_rows_kernel<DT::F16>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, rows, K, q, s);
  WMX_HIP(hipGetLastError());
}

// ---------------- 8-bit decoder weights (fp8 decode, model dtype MX8): one wave per weight row ----------------
// e = mx8_exp(max |row|) (the OCP MX rule with the block = the whole K row), q = RNE e4m3(w / 2^e) in the
// packed8_index layout, scale[n] = 2^e; rm (optional) = the dequantized row-major 16-bit copy (exact: an e4m3 value
// times a power of two is a bf16 / f16 value), which the many-row passes (prefill, alignment) run on so that every
// pass of the fp8 model sees the same weights.  oracle/whisper_np.py w8_rows restates the rule.
template <DT T>
__global__ __launch_bounds__(256) void w8_quantize_kernel(const uint16_t* __restrict__ src, int N, int Np, int K,
                                                          uint8_t* __restrict__ q8, float* __restrict__ scale,
                                                          uint16_t* __restrict__ rm) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= Np) return;  // (wave-uniform)
  float am = 0.f;
  for (int k = 8 * lane; k < K; k += 512) {
    const u16x8 h = *reinterpret_cast<const u16x8*>(src + packed_index(n, k, K));
#pragma unroll
    for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(to_f32<T>(h[e])));
  }
  am = wave_max(am);
  const int ex = mx8_exp(am);
  const float is = mx8_inv_scale(ex), sc = __int_as_float((127 + ex) << 23);
  for (int k = 8 * lane; k < K; k += 512) {
    const u16x8 h = *reinterpret_cast<const u16x8*>(src + packed_index(n, k, K));
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = to_f32<T>(h[e]) * is;
    const uint2 b = make_uint2(mx8_pack4(v[0], v[1], v[2], v[3]), mx8_pack4(v[4], v[5], v[6], v[7]));
    *reinterpret_cast<uint2*>(q8 + packed8_index(n, k, K)) = b;
    if (rm && n < N) {
      const u16x8 d = fp8x8_to16<T>(b.x, b.y);
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = from_f32<T>(to_f32<T>(d[e]) * sc);
      *reinterpret_cast<u16x8*>(rm + (long)n * K + k) = o;
    }
  }
  if (lane == 0) scale[n] = n < N ? sc : 0.f;
}

void launch_w8_quantize(DT dt, const uint16_t* src, int N, int K, uint8_t* q8, float* scale, uint16_t* rm,
                        hipStream_t st) {
  WMX_CHECK(K % 64 == 0 && N >= 1, "w8 quantize: K must be a multiple of 64");
  const int Np = (N + 15) / 16 * 16;
  if (dt == DT::BF16)
    hipLaunchKernelGGL(w8_quantize_kernel<DT::BF16>, dim3(cdiv(Np, 4)), dim3(256), 0, st, src, N, Np, K, q8, scale, rm);
  else
    hipLaunchKernelGGL(w8_quantize_kernel<DT::F16>, dim3(cdiv(Np, 4)), dim3(256), 0, st, src, N, Np, K, q8, scale, rm);
  WMX_HIP(hipGetLastError());
}

// ---------------- the CTranslate2 int8 grid (model dtype I8) ----------------
// One wave per weight row n of a packed 16-bit [N][K] matrix: the CT2 row scale s = 127 / max|w| (1 for an all-zero
// row; CTranslate2's int8 quantization, oracle/whisper_np.py int8_rows) written to ct2s[n] where ct2s[n] is 0 (not
// given), else ct2s[n] read as given (a CT2 int8 checkpoint's own weight_scale).  The given / derived state is the
// scale array itself, which lives in the broadcast parameter region: a rank that receives the arena keeps the
// sender's scales bit for bit.
// from it (a CT2 int8 checkpoint's own weight_scale); q = rint(w s) clamped to [-127, 127] as int8 bytes in the
// packed8_index layout, the GEMM's row multiplier 1 / s, and the row-major copy q / s rounded to 16 bits.  With the
// 16-bit weight w = round16(q_ckpt / s_ckpt) and the checkpoint's scale, |q_ckpt| <= 127 makes rint(w s) = q_ckpt
// exactly (the relative rounding of w is <= 2^-9, so |w s - q_ckpt| <= 127 / 512 < 1/2).
template <DT T>
__global__ __launch_bounds__(256) void i8_quantize_kernel(const uint16_t* __restrict__ src, int N, int Np, int K,
                                                          float* __restrict__ ct2s, uint8_t* __restrict__ q8,
                                                          float* __restrict__ mult, uint16_t* __restrict__ rm) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= Np) return;  // (wave-uniform)
  float s = 1.f;
  if (n < N) {
    s = ct2s[n];
    if (!(s > 0.f)) {  // (wave-uniform) not given: CT2's rule
      float am = 0.f;
      for (int k = 8 * lane; k < K; k += 512) {
        const u16x8 h = *reinterpret_cast<const u16x8*>(src + packed_index(n, k, K));
#pragma unroll
        for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(to_f32<T>(h[e])));
      }
      am = wave_max(am);
      s = am > 0.f ? 127.f / am : 1.f;
      if (lane == 0) ct2s[n] = s;
    }
  }
  for (int k = 8 * lane; k < K; k += 512) {
    uint32_t b[2] = {0u, 0u};
    u16x8 o;
    if (n < N) {
      const u16x8 h = *reinterpret_cast<const u16x8*>(src + packed_index(n, k, K));
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float q = fminf(127.f, fmaxf(-127.f, rintf(to_f32<T>(h[e]) * s)));
        b[e >> 2] |= (uint32_t)((int)q & 0xff) << (8 * (e & 3));
        o[e] = from_f32<T>(q / s);
      }
    }
    *reinterpret_cast<uint2*>(q8 + packed8_index(n, k, K)) = make_uint2(b[0], b[1]);
    if (rm && n < N) *reinterpret_cast<u16x8*>(rm + (long)n * K + k) = o;
  }
  if (lane == 0) mult[n] = n < N ? 1.f / s : 0.f;
}

void launch_i8_quantize(DT dt, const uint16_t* src, int N, int K, float* ct2s, uint8_t* q8, float* mult, uint16_t* rm,
                        hipStream_t st) {
  WMX_CHECK(K % 64 == 0 && N >= 1, "int8 quantize: K must be a multiple of 64");
  const int Np = (N + 15) / 16 * 16;
  if (dt == DT::BF16)
    hipLaunchKernelGGL(i8_quantize_kernel<DT::BF16>, dim3(cdiv(Np, 4)), dim3(256), 0, st, src, N, Np, K, ct2s,
                       q8, mult, rm);
  else
    hipLaunchKernelGGL(i8_quantize_kernel<DT::F16>, dim3(cdiv(Np, 4)), dim3(256), 0, st, src, N, Np, K, ct2s,
                       q8, mult, rm);
  WMX_HIP(hipGetLastError());
}

// ---------------- fp8 cross K / V^T images (fp8 decode): one 1024-thread workgroup per (layer-kv, window, head) image ---
// The image (192 KB of 16-bit values) is read ONCE into registers: wave w owns the fp8 piece blocks blk = w + 16 i
// (94 blocks of 64 pieces), and lane l loads the two 16-bit pieces (2 blk + hh) 64 + l, hh = 0, 1, that fp8 piece
// blk 64 + l is packed from (12 pieces of 16 B per thread).  The image amax is reduced over the workgroup -> e =
// mx8_exp (one power-of-two scale per image), then each lane packs and stores its pieces.  The zero pad keys stay zero.
// oracle/whisper_np.py kv8_images restates the rule.
template <DT T>
__global__ __launch_bounds__(1024) void crosskv_quant_kernel(const uint16_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                             float* __restrict__ scale, int xw, int H) {
  constexpr int kPieces = kXS * 64 / 16;  // fp8 pieces of one image (6016 = 94 blocks of 64)
  constexpr int kIt = (kPieces / 64 + 15) / 16;  // blocks per wave (16 waves): 6
  const int h = blockIdx.x, w = blockIdx.y, z = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long img = ((long)z * xw + w) * H + h;
  const u16x8* s = reinterpret_cast<const u16x8*>(src + img * kXS * 64);
  u16x8 a[kIt], b[kIt];
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int blk = wave + 16 * i;
    const bool ok = blk < kPieces / 64;
    const long p0 = 2L * min(blk, kPieces / 64 - 1) * 64 + lane;
    a[i] = s[p0];
    b[i] = s[p0 + 64];
    if (ok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fmaxf(fabsf(to_f32<T>(a[i][e])), fabsf(to_f32<T>(b[i][e]))));
    }
  }
  __shared__ float red[16];
  am = wave_max(am);
  if (lane == 0) red[wave] = am;
  __syncthreads();
  am = red[0];
#pragma unroll
  for (int k = 1; k < 16; ++k) am = fmaxf(am, red[k]);
  const int ex = mx8_exp(am);
  const float is = mx8_inv_scale(ex);
  uint8_t* d = dst + img * kXS * 64;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int blk = wave + 16 * i;
    if (blk >= kPieces / 64) break;  // (wave-uniform)
    u32x4 o;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      o[q] = mx8_pack4(to_f32<T>(a[i][4 * q]) * is, to_f32<T>(a[i][4 * q + 1]) * is, to_f32<T>(a[i][4 * q + 2]) * is,
                       to_f32<T>(a[i][4 * q + 3]) * is);
      o[2 + q] = mx8_pack4(to_f32<T>(b[i][4 * q]) * is, to_f32<T>(b[i][4 * q + 1]) * is,
                           to_f32<T>(b[i][4 * q + 2]) * is, to_f32<T>(b[i][4 * q + 3]) * is);
    }
    *reinterpret_cast<u32x4*>(d + ((long)blk * 64 + lane) * 16) = o;
  }
  if (tid == 0) scale[img] = __int_as_float((127 + ex) << 23);
}

void launch_crosskv_quant(const uint16_t* src, uint8_t* dst, float* scale, int L2, int xw, int B, int H,
                          hipStream_t st) {
  WMX_CHECK(B >= 1 && B <= xw && L2 >= 1 && H >= 1, "cross K/V quantize: shape");
  static_assert(kXS * 64 / 16 % 64 == 0, "whole 64-piece blocks per image");
  hipLaunchKernelGGL(crosskv_quant_kernel<DT::BF16>, dim3(H, B, L2), dim3(1024), 0, st, src, dst, scale, xw, H);
  WMX_HIP(hipGetLastError());
}

// ---------------- conv1 im2col: out[b*3000+t][kk*M + c] = mel[b][c][t+kk-1] (0 outside / in the K pad) ----------------
template <DT T>
__global__ __launch_bounds__(256) void im2col1_kernel(const float* __restrict__ mel, int B, int M, int Kp,
                                                      uint16_t* __restrict__ out) {
  // tile: 64 frames x all channels of one window, transposed through LDS for coalesced reads and writes
  __shared__ float tile[128][67];
  const int b = blockIdx.y, t0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  for (int i = tid; i < M * 66; i += 256) {  // channels x frames t0-1 .. t0+64
    const int cc = i / 66, tt = t0 - 1 + i % 66;
    tile[cc][i % 66] = (tt >= 0 && tt < 3000) ? mel[((long)b * M + cc) * 3000 + tt] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < 64 * Kp; i += 256) {
    const int tl = i / Kp, col = i % Kp;
    const int t = t0 + tl;
    if (t >= 3000) continue;
    float v = 0.f;
    if (col < 3 * M) {
      const int kk = col / M, c = col % M;
      v = tile[c][tl + kk];
    }
    out[((long)b * 3000 + t) * Kp + col] = from_f32<T>(v);
  }
}

void launch_im2col_conv1(DT dt, const float* mel, int B, int n_mels, int Kp, uint16_t* out, hipStream_t st) {
  WMX_CHECK(n_mels <= 128, "im2col1: n_mels");
  dim3 grid(cdiv(3000, 64), B);
  if (dt == DT::BF16)
    hipLaunchKernelGGL(im2col1_kernel<DT::BF16>, grid, dim3(256), 0, st, mel, B, n_mels, Kp, out);
  else
    hipLaunchKernelGGL(im2col1_kernel<DT::F16>, grid, dim3(256), 0, st, mel, B, n_mels, Kp, out);
  WMX_HIP(hipGetLastError());
}

// ---------------- conv2 im2col (stride 2): out[b*1500+t][kk*d + c] = h1[b*3000 + 2t+kk-1][c] ----------------
__global__ __launch_bounds__(256) void im2col2_kernel(const uint16_t* __restrict__ h1, int B, int d,
                                                      uint16_t* __restrict__ out) {
  const int n8 = d / 8;
  const long total = (long)B * 1500 * 3 * n8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c8 = (int)(i % n8);
    const long r = i / n8;
    const int kk = (int)(r % 3);
    const long bt = r / 3;
    const int t = (int)(bt % 1500), b = (int)(bt / 1500);
    const int ts = 2 * t + kk - 1;
    u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (ts >= 0 && ts < 3000) v = reinterpret_cast<const u16x8*>(h1 + ((long)b * 3000 + ts) * d)[c8];
    reinterpret_cast<u16x8*>(out + bt * 3 * d + kk * d)[c8] = v;
  }
}

void launch_im2col_conv2(DT, const uint16_t* h1, int B, int d, uint16_t* out, hipStream_t st) {
  const long total = (long)B * 1500 * 3 * (d / 8);
  hipLaunchKernelGGL(im2col2_kernel, dim3((int)std::min<long>((total + 255) / 256, 8192)), dim3(256), 0, st, h1, B, d,
                     out);
  WMX_HIP(hipGetLastError());
}

template <DT T>
__global__ void cvt_kernel(const uint16_t* __restrict__ in, float* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = to_f32<T>(in[i]);
}
void launch_cvt16_to_f32(DT dt, const uint16_t* in, float* out, long n, hipStream_t st) {
  dim3 g((int)std::min<long>((n + 255) / 256, 8192));
  if (dt == DT::BF16)
    hipLaunchKernelGGL(cvt_kernel<DT::BF16>, g, dim3(256), 0, st, in, out, n);
  else
    hipLaunchKernelGGL(cvt_kernel<DT::F16>, g, dim3(256), 0, st, in, out, n);
  WMX_HIP(hipGetLastError());
}

// ---------------- token + learned position embedding into the fp32 residual stream ----------------
template <DT T>
__global__ __launch_bounds__(256) void embed_kernel(const uint16_t* __restrict__ tok_emb, const uint16_t* __restrict__ pos_emb,
                                                    const int* __restrict__ hist, long hist_ld, int Tn,
                                                    const int* __restrict__ pad, const int* __restrict__ slot0, int d,
                                                    float* __restrict__ x, int V) {
  const int m = blockIdx.x;
  const int r = m / Tn, i = m - r * Tn;
  const int slot = *slot0 + i;
  // (clamped into the table: a token id is never an address outside it, whatever reached the history)
  const int tok = min(max(hist[(long)r * hist_ld + slot], 0), V - 1);
  int pos = slot - (pad ? pad[r] : 0);
  pos = max(pos, 0);
  for (int c = threadIdx.x; c < d; c += 256)
    x[(long)m * d + c] = to_f32<T>(tok_emb[packed_index(tok, c, d)]) + to_f32<T>(pos_emb[(long)pos * d + c]);
}

void launch_embed(DT dt, const uint16_t* tok_emb, const uint16_t* pos_emb, const int* hist, long hist_ld, int R, int Tn,
                  const int* pad, const int* slot0, int d, float* x, hipStream_t st, int V) {
  if (dt == DT::BF16)
    hipLaunchKernelGGL(embed_kernel<DT::BF16>, dim3(R * Tn), dim3(256), 0, st, tok_emb, pos_emb, hist, hist_ld, Tn, pad,
                       slot0, d, x, V);
  else
    hipLaunchKernelGGL(embed_kernel<DT::F16>, dim3(R * Tn), dim3(256), 0, st, tok_emb, pos_emb, hist, hist_ld, Tn, pad,
                       slot0, d, x, V);
  WMX_HIP(hipGetLastError());
}

// ---------------- row-major copy of a packed [N][K] matrix (packed_index) ----------------
__global__ __launch_bounds__(256) void unpack_packed_kernel(const uint16_t* __restrict__ p, uint16_t* __restrict__ rm,
                                                            int N, int K) {
  const long n8 = (long)N * K / 8;  // 8 consecutive k of a row are 8 consecutive packed elements (16 B)
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    const long n = e / K, k = e - n * K;
    *reinterpret_cast<u16x8*>(rm + e) = *reinterpret_cast<const u16x8*>(p + packed_index(n, k, K));
  }
}

void launch_unpack_packed(const uint16_t* packed, uint16_t* rowmajor, int N, int K, hipStream_t st) {
  WMX_CHECK(K % 32 == 0, "unpack: K must be a multiple of 32");
  hipLaunchKernelGGL(unpack_packed_kernel, dim3(2048), dim3(256), 0, st, packed, rowmajor, N, K);
  WMX_HIP(hipGetLastError());
}

// ---------------- decode step: token + position embedding and the first layer's LN1 in one launch ----------------
// one wave per row (4 rows per workgroup); the same arithmetic as embed_kernel followed by layernorm_kernel
// stats != null (LayerNorm folded into the projections): out = the 16-bit copy of x, stats[g][r] = (mean, M2) of
// each aligned 16-column group g of x (wmx_common.h row_ln_from_stats), no LN here
template <DT T>
__global__ __launch_bounds__(256) void embed_ln_kernel(const uint16_t* __restrict__ tok_emb,
                                                       const uint16_t* __restrict__ pos_emb, const int* __restrict__ hist,
                                                       long hist_ld, const int* __restrict__ pad,
                                                       const int* __restrict__ slot0, const float* __restrict__ g,
                                                       const float* __restrict__ bb, int rows, int d,
                                                       float* __restrict__ x, uint16_t* __restrict__ out,
                                                       float2* __restrict__ stats, long stats_ld, int V) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const int slot = *slot0;
  const int tok = min(max(hist[(long)r * hist_ld + slot], 0), V - 1);  // (clamped into the table, as embed_kernel)
  const int pos = max(slot - (pad ? pad[r] : 0), 0);
  const int n4 = d >> 2;
  float4 v[8];  // d <= 2048
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + i * 64;
    if (c < n4) {
      // four consecutive k of one packed row are contiguous (packed_index keeps k & 7 innermost)
      const u16x4 te = *reinterpret_cast<const u16x4*>(tok_emb + packed_index(tok, 4 * c, d));
      const u16x4 pe = *reinterpret_cast<const u16x4*>(pos_emb + (long)pos * d + 4 * c);
      v[i] = make_float4(to_f32<T>(te[0]) + to_f32<T>(pe[0]), to_f32<T>(te[1]) + to_f32<T>(pe[1]),
                         to_f32<T>(te[2]) + to_f32<T>(pe[2]), to_f32<T>(te[3]) + to_f32<T>(pe[3]));
      reinterpret_cast<float4*>(x + (long)r * d)[c] = v[i];
      s += v[i].x + v[i].y + v[i].z + v[i].w;
    } else {
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if (stats) {  // per 16-column group = 4 consecutive quads = an aligned group of 4 lanes (d % 64 == 0)
    uint16_t* o = out + (long)r * d;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i * 64 >= n4) break;  // wave-uniform
      const int c = lane + i * 64;
      const float4 a = v[i];
      const float mg = sum4_lanes((a.x + a.y) + (a.z + a.w)) * (1.f / 16.f);
      const float dx = a.x - mg, dy = a.y - mg, dz = a.z - mg, dw = a.w - mg;
      const float m2 = sum4_lanes((dx * dx + dy * dy) + (dz * dz + dw * dw));
      if (c < n4) {
        const u16x4 h = {from_f32<T>(a.x), from_f32<T>(a.y), from_f32<T>(a.z), from_f32<T>(a.w)};
        reinterpret_cast<u16x4*>(o)[c] = h;
        if ((c & 3) == 0) stats[(long)(c >> 2) * stats_ld + r] = make_float2(mg, m2);
      }
    }
    return;
  }
  const float mean = wave_sum(s) / d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + i * 64;
    if (c < n4) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, e = v[i].w - mean;
      q += a * a + b * b + cc * cc + e * e;
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / d + 1e-5f);
  uint16_t* o = out + (long)r * d;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + i * 64;
    if (c < n4) {
      const float4 gg = reinterpret_cast<const float4*>(g)[c];
      const float4 be = reinterpret_cast<const float4*>(bb)[c];
      u16x4 w;
      w[0] = from_f32<T>((v[i].x - mean) * rstd * gg.x + be.x);
      w[1] = from_f32<T>((v[i].y - mean) * rstd * gg.y + be.y);
      w[2] = from_f32<T>((v[i].z - mean) * rstd * gg.z + be.z);
      w[3] = from_f32<T>((v[i].w - mean) * rstd * gg.w + be.w);
      reinterpret_cast<u16x4*>(o)[c] = w;
    }
  }
}

void launch_embed_ln(DT dt, const uint16_t* tok_emb, const uint16_t* pos_emb, const int* hist, long hist_ld, int R,
                     const int* pad, const int* slot0, const float* g, const float* b, int d, float* x, uint16_t* out,
                     hipStream_t st, int V, float2* stats, long stats_ld) {
  WMX_CHECK(d % 32 == 0 && d <= 2048 && (!stats || d % 64 == 0) && V >= 1, "embed_ln: d");
  dim3 grid(cdiv(R, 4));
  if (dt == DT::BF16)
    hipLaunchKernelGGL(embed_ln_kernel<DT::BF16>, grid, dim3(256), 0, st, tok_emb, pos_emb, hist, hist_ld, pad, slot0,
                       g, b, R, d, x, out, stats, stats_ld, V);
  else
    hipLaunchKernelGGL(embed_ln_kernel<DT::F16>, grid, dim3(256), 0, st, tok_emb, pos_emb, hist, hist_ld, pad, slot0,
                       g, b, R, d, x, out, stats, stats_ld, V);
  WMX_HIP(hipGetLastError());
}

// ---------------- LayerNorm folded into the following projection (decode step; wmx_common.h) ----------------
// one workgroup per output row n of W [N][K] (row-major copy): Wp (packed) = 16-bit(W[n][k] g[k]),
// c1[n] = sum_k Wp[n][k] (the rounded values the GEMM multiplies), c2[n] = bias[n] + sum_k b[k] W[n][k]
template <DT T>
__global__ __launch_bounds__(256) void fold_ln_kernel(const uint16_t* __restrict__ Wrm, const float* __restrict__ g,
                                                      const float* __restrict__ b, const float* __restrict__ bias,
                                                      int K, uint16_t* __restrict__ Wp, float* __restrict__ c1,
                                                      float* __restrict__ c2, int rowmajor) {
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float red[2][4];
  float s1 = 0.f, s2 = 0.f;
  for (int k = tid; k < K; k += 256) {
    const float w = to_f32<T>(Wrm[(long)n * K + k]);
    const uint16_t wf = from_f32<T>(w * g[k]);
    Wp[rowmajor ? (long)n * K + k : packed_index(n, k, K)] = wf;
    s1 += to_f32<T>(wf);
    s2 += b[k] * w;
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    red[0][wave] = s1;
    red[1][wave] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    c1[n] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    c2[n] = (bias ? bias[n] : 0.f) + ((red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
  }
}

void launch_fold_ln(DT dt, const uint16_t* Wrm, const float* g, const float* b, const float* bias, int N, int K,
                    uint16_t* Wp, float* c1, float* c2, hipStream_t st, bool rowmajor) {
  WMX_CHECK(N % 16 == 0 && K % 32 == 0, "fold_ln: shape");
  const int rm = rowmajor ? 1 : 0;
  if (dt == DT::BF16)
    hipLaunchKernelGGL(fold_ln_kernel<DT::BF16>, dim3(N), dim3(256), 0, st, Wrm, g, b, bias, K, Wp, c1, c2, rm);
  else
    hipLaunchKernelGGL(fold_ln_kernel<DT::F16>, dim3(N), dim3(256), 0, st, Wrm, g, b, bias, K, Wp, c1, c2, rm);
  WMX_HIP(hipGetLastError());
}

// ---------------- split-K reduction + residual + LayerNorm (decode step) ----------------
// one 1024-thread workgroup per row: every partial slice of the thread's columns is loaded in one batch (slice
// order kept in the sum), v = x + bias + sum_s part[s], x = v, out16 = LN(v) * g + b
constexpr int kRedThreads = 1024, kRedMaxS = 8;
template <DT T>
__global__ __launch_bounds__(kRedThreads) void reduce_ln_kernel(const float* __restrict__ part, int S, long pstride,
                                                                const float* __restrict__ bias, float* __restrict__ x,
                                                                const float* __restrict__ g, const float* __restrict__ b,
                                                                uint16_t* __restrict__ out, int d) {
  // (not probed: the float4 form below is the one the decode step runs)
  constexpr int MAXV = 2;  // d <= 2048
  constexpr int NW = kRedThreads / 64;
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float red[2][NW];
  float t[MAXV][kRedMaxS], xv[MAXV], bv[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = tid + i * kRedThreads;
    const bool ok = c < d;
    xv[i] = ok ? x[(long)m * d + c] : 0.f;
    bv[i] = ok && bias ? bias[c] : 0.f;
#pragma unroll
    for (int u = 0; u < kRedMaxS; ++u) t[i][u] = (ok && u < S) ? part[u * pstride + (long)m * d + c] : 0.f;
  }
  float v[MAXV];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    float p = 0.f;
#pragma unroll
    for (int u = 0; u < kRedMaxS; ++u) p += t[i][u];
    const int c = tid + i * kRedThreads;
    v[i] = 0.f;
    if (c < d) {
      v[i] = xv[i] + bv[i] + p;
      x[(long)m * d + c] = v[i];
      sum += v[i];
    }
  }
  if (!g) return;
  sum = wave_sum(sum);
  if (lane == 0) red[0][wave] = sum;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w2 = 0; w2 < NW; ++w2) tot += red[0][w2];
  const float mean = tot / d;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = tid + i * kRedThreads;
    if (c < d) {
      const float q = v[i] - mean;
      sq += q * q;
    }
  }
  sq = wave_sum(sq);
  if (lane == 0) red[1][wave] = sq;
  __syncthreads();
  float tq = 0.f;
#pragma unroll
  for (int w2 = 0; w2 < NW; ++w2) tq += red[1][w2];
  const float rstd = 1.0f / sqrtf(tq / d + 1e-5f);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = tid + i * kRedThreads;
    if (c < d) out[(long)m * d + c] = from_f32<T>((v[i] - mean) * rstd * g[c] + b[c]);
  }
}

// float4 form (d % 4 == 0, d <= 4096): one thread per column quad (d / 4 threads rounded up to whole waves, 320
// for large-v3), all S + 2 quads of the thread loaded in one batch; fewer, wider loads and 5 waves instead of 16
// in the two block reductions, which is what this latency-bound step pays for
template <DT T>
__global__ __launch_bounds__(1024) void reduce_ln4_kernel(const float* __restrict__ part, int S, long pstride,
                                                          const float* __restrict__ bias, float* __restrict__ x,
                                                          const float* __restrict__ g, const float* __restrict__ b,
                                                          uint16_t* __restrict__ out, int d,
                                                          unsigned long long* __restrict__ tprobe,
                                                          const int* __restrict__ pslot) {
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const unsigned long long probe_t0 = (tprobe && tid == 0) ? probe_clock() : 0ull;  // in-situ probe
  __shared__ float red[2][16];
  const int c = tid * 4;
  const bool ok = c < d;
  float4 t[kRedMaxS], xv = make_float4(0.f, 0.f, 0.f, 0.f), bv = xv, gg = xv, bb = xv;
  if (ok) {
    xv = *reinterpret_cast<const float4*>(x + (long)m * d + c);
    if (bias) bv = *reinterpret_cast<const float4*>(bias + c);
    if (g) {  // the LayerNorm parameters ride in the same load batch (not a second round trip after the reductions)
      gg = *reinterpret_cast<const float4*>(g + c);
      bb = *reinterpret_cast<const float4*>(b + c);
    }
  }
#pragma unroll
  for (int u = 0; u < kRedMaxS; ++u)
    t[u] = (ok && u < S) ? *reinterpret_cast<const float4*>(part + u * pstride + (long)m * d + c)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < kRedMaxS; ++u) p = make_float4(p.x + t[u].x, p.y + t[u].y, p.z + t[u].z, p.w + t[u].w);
  const float4 v = make_float4(xv.x + bv.x + p.x, xv.y + bv.y + p.y, xv.z + bv.z + p.z, xv.w + bv.w + p.w);
  if (ok) *reinterpret_cast<float4*>(x + (long)m * d + c) = v;
  if (!g) {
    if (tprobe && tid == 0) probe_record(tprobe, *pslot, probe_t0);
    return;
  }
  float sum = ok ? (v.x + v.y) + (v.z + v.w) : 0.f;
  sum = wave_sum(sum);
  if (lane == 0) red[0][wave] = sum;
  __syncthreads();
  float tot = 0.f;
  for (int w2 = 0; w2 < nw; ++w2) tot += red[0][w2];
  const float mean = tot / d;
  const float4 q = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
  float sq = ok ? (q.x * q.x + q.y * q.y) + (q.z * q.z + q.w * q.w) : 0.f;
  sq = wave_sum(sq);
  if (lane == 0) red[1][wave] = sq;
  __syncthreads();
  float tq = 0.f;
  for (int w2 = 0; w2 < nw; ++w2) tq += red[1][w2];
  const float rstd = 1.0f / sqrtf(tq / d + 1e-5f);
  if (ok) {
    const u16x4 h = {from_f32<T>(q.x * rstd * gg.x + bb.x), from_f32<T>(q.y * rstd * gg.y + bb.y),
                     from_f32<T>(q.z * rstd * gg.z + bb.z), from_f32<T>(q.w * rstd * gg.w + bb.w)};
    *reinterpret_cast<u16x4*>(out + (long)m * d + c) = h;
  }
  if (tprobe && tid == 0) probe_record(tprobe, *pslot, probe_t0);
}

void launch_reduce_ln(DT dt, const float* part, int S, const float* bias, float* x, const float* g, const float* b,
                      uint16_t* out16, int rows, int d, hipStream_t st, unsigned long long* tprobe,
                      const int* pslot) {
  WMX_CHECK(d <= 2 * kRedThreads && S >= 1 && S <= kRedMaxS, "reduce_ln: width / split count");
  const long pstride = (long)rows * d;
  if (d % 4 == 0 && d <= 4096) {
    const int nt = ((d / 4 + 63) / 64) * 64;
    if (dt == DT::BF16)
      hipLaunchKernelGGL(reduce_ln4_kernel<DT::BF16>, dim3(rows), dim3(nt), 0, st, part, S, pstride, bias, x, g, b,
                         out16, d, tprobe, pslot);
    else
      hipLaunchKernelGGL(reduce_ln4_kernel<DT::F16>, dim3(rows), dim3(nt), 0, st, part, S, pstride, bias, x, g, b,
                         out16, d, tprobe, pslot);
    WMX_HIP(hipGetLastError());
    return;
  }
  if (dt == DT::BF16)
    hipLaunchKernelGGL(reduce_ln_kernel<DT::BF16>, dim3(rows), dim3(kRedThreads), 0, st, part, S, pstride, bias, x, g,
                       b, out16, d);
  else
    hipLaunchKernelGGL(reduce_ln_kernel<DT::F16>, dim3(rows), dim3(kRedThreads), 0, st, part, S, pstride, bias, x, g,
                       b, out16, d);
  WMX_HIP(hipGetLastError());
}

// ---------------- synthetic weights: u = splitmix64(seed*G1 + tid*G2 + i) top 24 bits -> [-1,1) ----------------
__device__ inline float prng_u(uint64_t key, uint64_t i) {
  uint64_t z = key + i;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  const float k = (float)(uint32_t)(z >> 40);
  return __fsub_rn(__fmul_rn(k, 1.1920928955078125e-7f), 1.0f);
}

template <DT T>
__global__ void init_kernel(uint64_t key, InitSpec s) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < s.n; i += (long)gridDim.x * 256) {
    float v = __fmul_rn(prng_u(key, (uint64_t)i), s.scale);
    if (s.offset != 0.f) v = __fadd_rn(v, s.offset);
    long di = i;
    if (s.kind == 1) {  // conv [O][C][3] -> [O][Kp] at kk*C + c
      const int kk = (int)(i % 3);
      const long oc = i / 3;
      const int c = (int)(oc % s.C);
      const long o = oc / s.C;
      di = o * s.Kp + (long)kk * s.C + c;
    } else if (s.kind == 2) {
      di = packed_index(i / s.Kp, i % s.Kp, s.Kp);
    }
    if (s.store_f32) {
      // f32 storage of a 16-bit parameter: keep the value the 16-bit storage would hold
      const uint16_t h = from_f32<T>(v);
      reinterpret_cast<float*>(s.dst)[di] = to_f32<T>(h);
    } else {
      reinterpret_cast<uint16_t*>(s.dst)[di] = from_f32<T>(v);
    }
  }
}

void launch_init_tensor(DT dt, uint64_t seed, const InitSpec& s, hipStream_t st) {
  const uint64_t key = seed * 0x9E3779B97F4A7C15ull + (uint64_t)s.tid * 0xBF58476D1CE4E5B9ull;
  dim3 g((int)std::min<long>((s.n + 255) / 256, 16384));
  if (dt == DT::BF16)
    hipLaunchKernelGGL(init_kernel<DT::BF16>, g, dim3(256), 0, st, key, s);
  else
    hipLaunchKernelGGL(init_kernel<DT::F16>, g, dim3(256), 0, st, key, s);
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Shader-clock probe (bench.py's encoder field, diagnostic): one wave per workgroup sleeps until `rt_ticks` of the
// 100 MHz constant clock have passed and reports the shader clock it ran at, d(s_memtime) / d(s_memrealtime) x
// 100 MHz (MI355X_MICROARCH.md 'DVFS give-back' item 6).  Launched beside a workload on a stream of its own; a
// deadline on the constant clock bounds every wave.  Workgroup i lands on XCD i mod 8.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void clock_probe_kernel(float* __restrict__ out, long long rt_ticks) {
  const long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
  long long r = r0;
  while (r - r0 < rt_ticks) {
    __builtin_amdgcn_s_sleep(127);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = (float)((double)(t1 - t0) / (double)(r - r0) * 100.0);
}

void launch_clock_probe(float* out, int n, double ms, hipStream_t st) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(n), dim3(64), 0, st, out, (long long)(ms * 1e5));
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
