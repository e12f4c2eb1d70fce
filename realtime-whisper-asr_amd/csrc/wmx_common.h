// Shared device helpers for libwmx (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <stdexcept>
#include <string>

namespace wmx {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

// Cache policy of the decode step's once-read streams (MI355X_MICROARCH.md "nt-weights"): WMX_WNT=1 loads the
// packed decoder weights non-temporally, WMX_KV_AUX=2 sets nt on the cross-K/V buffer loads.  Build-time
// switches for A/B runs (tools/build_variant.sh); the defaults are what was measured fastest.
#ifndef WMX_WNT
#define WMX_WNT 0
#endif
#ifndef WMX_KV_AUX
#define WMX_KV_AUX 0
#endif
template <class V>
__device__ inline V stream_load(const V* p) {
  if constexpr (WMX_WNT) return __builtin_nontemporal_load(p);
  else return *p;
}

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define WMX_HIP(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      throw ::wmx::Error(2, std::string(#expr) + ": " + hipGetErrorString(e_) + " @" __FILE__ ":" + \
                         std::to_string(__LINE__));                                             \
  } while (0)

#define WMX_CHECK(cond, msg)                                 \
  do {                                                       \
    if (!(cond)) throw ::wmx::Error(1, std::string(msg));    \
  } while (0)

// ---- 16-bit storage types: bf16 and f16 share uint16_t storage; conversions are explicit ----
enum class DT { BF16 = 0, F16 = 1 };

__device__ __host__ inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
// round-to-nearest-even (same formula as oracle.round_bf16; inputs are never NaN here)
__device__ __host__ inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ inline float f16_to_f32(uint16_t h) {
  _Float16 v;
  __builtin_memcpy(&v, &h, 2);
  return (float)v;
}
__device__ inline uint16_t f32_to_f16(float f) {
  _Float16 v = (_Float16)f;
  uint16_t h;
  __builtin_memcpy(&h, &v, 2);
  return h;
}

template <DT T> __device__ inline float to_f32(uint16_t h);
template <> __device__ inline float to_f32<DT::BF16>(uint16_t h) { return bf16_to_f32(h); }
template <> __device__ inline float to_f32<DT::F16>(uint16_t h) { return f16_to_f32(h); }
template <DT T> __device__ inline uint16_t from_f32(float f);
// the hardware round-to-nearest-even convert (v_cvt_pk_bf16_f32): bit-identical to f32_to_bf16 for non-NaN input
template <> __device__ inline uint16_t from_f32<DT::BF16>(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
template <> __device__ inline uint16_t from_f32<DT::F16>(float f) { return f32_to_f16(f); }

// MFMA 16x16x32 on 8 x 16-bit operands held as u16x8
template <DT T> __device__ inline f32x4 mfma16(const u16x8& a, const u16x8& b, f32x4 c);
template <> __device__ inline f32x4 mfma16<DT::BF16>(const u16x8& a, const u16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <> __device__ inline f32x4 mfma16<DT::F16>(const u16x8& a, const u16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// exact-erf GELU (Whisper's nn.GELU()).  erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the
// bf16/f16 rounding of every GELU output here): one exp, one reciprocal and five FMAs instead of ocml erff,
// which cost the encoder's fc1 epilogue ~50 us per layer at large-v3 x 8 windows.
__device__ inline float erf_fast(float z) {
  const float a = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float r = 1.0f - p * t * __expf(-a * a);
  return copysignf(r, z);
}
// gelu(x) = x Phi(x), Phi(x) = 1 - Q(|x|) for x >= 0 and Q(|x|) for x < 0, with Q(a) = 0.5 erfc(a / sqrt 2) from the
// same A&S 7.1.26 expansion as erf_fast, its constants pre-scaled (1 / sqrt 2 folded into t, 0.5 into the
// polynomial, log2(e) / 2 into the exponent): 15 VALU ops (2 transcendental) instead of ~19
// Load of a launch-uniform int that no wave of this launch writes (decode slot, row padding) through the scalar
// data cache: s_load_dword, waited by lgkmcnt, so it does not order behind (or in front of) the vector loads of the
// kernel's first batch, and the value is scalar without a readfirstlane.  Read-only use: the scalar cache is
// invalidated at every dispatch, so the previous launch's stores are seen.
__device__ __forceinline__ int load_uniform_i32(const int* p) {
  typedef const __attribute__((address_space(4))) int cint4;
  return *(cint4*)p;
}

// the same GELU on two values with packed f32 math (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth per issue, for
// epilogues that run outside any MFMA shadow); the transcendental and select steps stay per element
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ inline f32x2 gelu_erf2(f32x2 x) {
  const f32x2 ax = __builtin_elementwise_abs(x);
  const f32x2 d = __builtin_elementwise_fma(ax, f32x2{0.3275911f * 0.70710678118654752f, 0.3275911f * 0.70710678118654752f},
                                            f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = __builtin_elementwise_fma(f32x2{0.5f * 1.061405429f, 0.5f * 1.061405429f}, t,
                                      f32x2{0.5f * -1.453152027f, 0.5f * -1.453152027f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.5f * 1.421413741f, 0.5f * 1.421413741f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.5f * -0.284496736f, 0.5f * -0.284496736f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.5f * 0.254829592f, 0.5f * 0.254829592f});
  const f32x2 e2 = x * (x * f32x2{-0.72134752044448170f, -0.72134752044448170f});
  const f32x2 q = p * t * f32x2{__builtin_amdgcn_exp2f(e2.x), __builtin_amdgcn_exp2f(e2.y)};
  const f32x2 phi = {x.x >= 0.f ? 1.0f - q.x : q.x, x.y >= 0.f ? 1.0f - q.y : q.y};
  return x * phi;
}
__device__ inline float4 gelu_erf4(float4 v) {
  const f32x2 a = gelu_erf2(f32x2{v.x, v.y}), b = gelu_erf2(f32x2{v.z, v.w});
  return make_float4(a.x, a.y, b.x, b.y);
}

__device__ inline float gelu_erf(float x) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(x), 1.0f));
  float p = fmaf(0.5f * 1.061405429f, t, 0.5f * -1.453152027f);
  p = fmaf(p, t, 0.5f * 1.421413741f);
  p = fmaf(p, t, 0.5f * -0.284496736f);
  p = fmaf(p, t, 0.5f * 0.254829592f);
  const float q = p * t * __builtin_amdgcn_exp2f(x * (x * -0.72134752044448170f));  // exp(-x^2 / 2)
  return x * (x >= 0.f ? 1.0f - q : q);
}

// ---- cross-lane reductions on DPP and permlane swaps (VALU latency, no LDS round trip as ds_bpermute has).
// Every lane of the wave must be active.  All lanes end with the bit-identical result (each step combines
// a value with its partner's, and + / max are commutative).
template <int CTRL>
__device__ inline float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1;      // quad_perm [1,0,3,2]: lane ^ 1
constexpr int kDppXor2 = 0x4E;      // quad_perm [2,3,0,1]: lane ^ 2
constexpr int kDppHalfMirror = 0x141;  // lane i <-> 7 - i within 8: the other quad of an 8-lane group
constexpr int kDppMirror = 0x140;   // lane i <-> 15 - i within 16: the other 8-lane group of a row
constexpr int kDppXor8 = 0x128;     // row_ror:8: lane ^ 8
// v + v[lane ^ 16] and v + v[lane ^ 32]: a permlane swap of (v, v) returns this lane's value and its partner's,
// in either order
__device__ inline float sum_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ inline float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ inline float max_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ inline float max_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// sum over each aligned group of 8 lanes
__device__ inline float sum8_lanes(float v) {
  v += dpp_mov<kDppXor1>(v);
  v += dpp_mov<kDppXor2>(v);
  return v + dpp_mov<kDppHalfMirror>(v);
}
// sum over each aligned group of 4 lanes
__device__ inline float sum4_lanes(float v) {
  v += dpp_mov<kDppXor1>(v);
  return v + dpp_mov<kDppXor2>(v);
}
__device__ inline float wave_sum(float v) {
  v = sum8_lanes(v);
  v += dpp_mov<kDppMirror>(v);
  return sum_xor32(sum_xor16(v));
}
__device__ inline float wave_max(float v) {
  v = fmaxf(v, dpp_mov<kDppXor1>(v));
  v = fmaxf(v, dpp_mov<kDppXor2>(v));
  v = fmaxf(v, dpp_mov<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_mov<kDppMirror>(v));
  return max_xor32(max_xor16(v));
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---- LayerNorm folded into the following projection (decode step) ----
// The producer of a residual row x (embedding, an unsplit projection epilogue) stores, per aligned group of 16
// columns g, (mean_g, M2_g = sum (x - mean_g)^2) at stats[g * ld + row].  The consumer merges the d / 16 groups
// (Chan et al.'s pairwise update for equal counts: mean = avg mean_g, M2 = sum M2_g + 16 sum (mean_g - mean)^2,
// i.e. sum (x - mean)^2 exactly) and applies LN through the folded weights:
//   LN(x) W^T + bias = rstd (x W'^T - mean c1) + c2,  W' = W diag(g),  c1 = W' 1,  c2 = bias + W b.
// One wave per row, every lane active; G = d / 16 <= 128.  Returns (mean, rstd).
// (split in two so a kernel can issue the statistics loads early and merge them where it needs the result)
__device__ inline void row_ln_stats_load(const float2* __restrict__ st, long ld, int G, float2& a, float2& b) {
  const int lane = threadIdx.x & 63;
  a = lane < G ? st[lane * ld] : make_float2(0.f, 0.f);
  b = lane + 64 < G ? st[(lane + 64) * ld] : make_float2(0.f, 0.f);
}
// (hardware reciprocal and reciprocal square root, not the IEEE division and sqrt expansions: with four waves per
// SIMD each merging two rows, those expansions were ~2 us of every LayerNorm-folded decode launch, round 6)
__device__ inline float2 row_ln_stats_merge(float2 a, float2 b, int G) {
  const int lane = threadIdx.x & 63;
  const float invG = __builtin_amdgcn_rcpf((float)G);
  const float mean = wave_sum(a.x + b.x) * invG;
  const float da = lane < G ? a.x - mean : 0.f, db = lane + 64 < G ? b.x - mean : 0.f;
  const float m2 = wave_sum((a.y + b.y) + 16.f * (da * da + db * db));
  return make_float2(mean, __builtin_amdgcn_rsqf(m2 * (0.0625f * invG) + 1e-5f));
}
// sum over each aligned half-wave (32 lanes)
__device__ inline float half_sum32(float v) {
  v = sum8_lanes(v);
  v += dpp_mov<kDppMirror>(v);
  return sum_xor16(v);
}
// two rows at once, one per half-wave (lanes 0..31 row A, 32..63 row B): the row's G <= 128 groups of a row-major
// [row][G] statistics image, four per lane (group (lane & 31) + 32 q); then each half's (mean, rstd).  Half the
// reduction chains of merging the rows one after the other with the whole wave.
__device__ inline void row_ln_stats_load2(const float2* __restrict__ ra, const float2* __restrict__ rb, int G,
                                          float2 (&s)[4]) {
  const int lane = threadIdx.x & 63, i = lane & 31;
  const float2* st = lane < 32 ? ra : rb;
#pragma unroll
  for (int q = 0; q < 4; ++q) s[q] = i + 32 * q < G ? st[i + 32 * q] : make_float2(0.f, 0.f);
}
__device__ inline float2 row_ln_stats_merge2(const float2 (&s)[4], int G) {
  const int i = threadIdx.x & 31;
  const float invG = __builtin_amdgcn_rcpf((float)G);
  const float mean = half_sum32((s[0].x + s[1].x) + (s[2].x + s[3].x)) * invG;
  float dev = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float d = i + 32 * q < G ? s[q].x - mean : 0.f;
    dev += s[q].y + 16.f * d * d;
  }
  const float m2 = half_sum32(dev);
  return make_float2(mean, __builtin_amdgcn_rsqf(m2 * (0.0625f * invG) + 1e-5f));
}
__device__ inline float2 row_ln_from_stats(const float2* __restrict__ st, long ld, int G) {
  float2 a, b;
  row_ln_stats_load(st, ld, G, a, b);
  return row_ln_stats_merge(a, b, G);
}

// ---- OCP MX-fp8: e4m3 elements (OCP "fn", max 448), one e8m0 scale 2^e per 32 consecutive K elements ----
// e = the smallest power of two with amax / 2^e <= 448, taken from the f32 bits of amax (amax = m 2^k with
// m in [0.5, 1): e = k - 9 + (m > 0.875)), clamped to [-126, 126]; the scale byte is e + 127.  Elements are
// x / 2^e rounded to nearest-even e4m3 by v_cvt_pk_fp8_f32 (tools/mx8_check.hip: bit-exact vs RNE on 2^16
// values).  oracle/whisper_np.py mx8_quantize restates the same rule.
__device__ __host__ inline int mx8_exp(float amax) {
  uint32_t u;
  __builtin_memcpy(&u, &amax, 4);
  const int E = (int)((u >> 23) & 255u), Mt = (int)(u & 0x7fffffu);
  const int e = E - 135 + (Mt > 0x600000 ? 1 : 0);
  return e < -126 ? -126 : (e > 126 ? 126 : e);
}
__device__ inline float mx8_inv_scale(int e) { return __int_as_float((127 - e) << 23); }  // 2^-e, exact
// eight e4m3 bytes (two dwords, little-endian) -> eight 16-bit MFMA operand values.  Exact: every e4m3 value is a
// bf16 and an f16 value (v_cvt_scalef32_pk_{bf16,f16}_fp8 with scale 1; the row / image scale is applied outside)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <DT T> __device__ inline u16x8 fp8x8_to16(uint32_t a, uint32_t b);
template <> __device__ inline u16x8 fp8x8_to16<DT::BF16>(uint32_t a, uint32_t b) {
  const u32x4 r = {__builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(a, 1.0f, false)),
                   __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(a, 1.0f, true)),
                   __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(b, 1.0f, false)),
                   __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(b, 1.0f, true))};
  return __builtin_bit_cast(u16x8, r);
}
template <> __device__ inline u16x8 fp8x8_to16<DT::F16>(uint32_t a, uint32_t b) {
  const u32x4 r = {__builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(a, 1.0f, false)),
                   __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(a, 1.0f, true)),
                   __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(b, 1.0f, false)),
                   __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(b, 1.0f, true))};
  return __builtin_bit_cast(u16x8, r);
}
// 16 e4m3 bytes of one lane -> the two 8-element operands they hold (bytes 0..7, bytes 8..15)
template <DT T> __device__ inline void fp8x16_to16(const u32x4& w, u16x8& lo, u16x8& hi) {
  lo = fp8x8_to16<T>(w[0], w[1]);
  hi = fp8x8_to16<T>(w[2], w[3]);
}

// int8 weights (the CTranslate2 int8 grid, model dtype I8): 8 signed bytes -> 8 exact 16-bit values (|x| <= 127 is
// exact in f16 and bf16; the row scale is applied outside, as for e4m3).  f16: the byte x + 128 placed under the
// exponent byte 0x64 is the f16 1024 + x + 128 (ulp 1 in [1024, 2048)), minus 1152 on the packed adder; bf16: under
// 0x4B it is the f32 2^23 + x + 128, minus 2^23 + 128, then rounded to bf16 (exact)
template <DT T> __device__ inline u16x8 i8x8_to16(uint32_t a, uint32_t b);
template <> __device__ inline u16x8 i8x8_to16<DT::F16>(uint32_t a, uint32_t b) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const uint32_t xa = a ^ 0x80808080u, xb = b ^ 0x80808080u;
  const h2 off = {(_Float16)-1152.0f, (_Float16)-1152.0f};
  const h2 r0 = __builtin_bit_cast(h2, __builtin_amdgcn_perm(0x64646464u, xa, 0x05010400u)) + off;
  const h2 r1 = __builtin_bit_cast(h2, __builtin_amdgcn_perm(0x64646464u, xa, 0x05030402u)) + off;
  const h2 r2 = __builtin_bit_cast(h2, __builtin_amdgcn_perm(0x64646464u, xb, 0x05010400u)) + off;
  const h2 r3 = __builtin_bit_cast(h2, __builtin_amdgcn_perm(0x64646464u, xb, 0x05030402u)) + off;
  const u32x4 r = {__builtin_bit_cast(uint32_t, r0), __builtin_bit_cast(uint32_t, r1), __builtin_bit_cast(uint32_t, r2),
                   __builtin_bit_cast(uint32_t, r3)};
  return __builtin_bit_cast(u16x8, r);
}
template <> __device__ inline u16x8 i8x8_to16<DT::BF16>(uint32_t a, uint32_t b) {
  const uint32_t x[2] = {a ^ 0x80808080u, b ^ 0x80808080u};
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t sel = 0x040c0c00u | (uint32_t)(e & 3);  // [byte e, 0, 0, 0x4B]
    const float f = __builtin_bit_cast(float, __builtin_amdgcn_perm(0x4B4B4B4Bu, x[e >> 2], sel)) - 8388736.0f;
    o[e] = from_f32<DT::BF16>(f);
  }
  return o;
}
// 16 int8 bytes of one lane -> the two 8-element operands they hold (bytes 0..7, bytes 8..15)
template <DT T> __device__ inline void i8x16_to16(const u32x4& w, u16x8& lo, u16x8& hi) {
  lo = i8x8_to16<T>(w[0], w[1]);
  hi = i8x8_to16<T>(w[2], w[3]);
}

// four values (already divided by the block scale) -> four e4m3 bytes, little-endian in one dword
__device__ inline uint32_t mx8_pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}
// max |x| over the 8 consecutive lanes of an aligned group (a 32-element block held 4 per lane)
__device__ inline float max8_lanes(float v) {
  v = fmaxf(v, __shfl_xor(v, 1));
  v = fmaxf(v, __shfl_xor(v, 2));
  v = fmaxf(v, __shfl_xor(v, 4));
  return v;
}

// in-situ launch probe (bench roofline): every workgroup of a probed launch stores its own [start, end] device
// wall-clock ticks at [slot][workgroup] with one plain 16-byte store (no shared counter to contend on); the host
// takes the min start / max end over the workgroups of a slot after the timed region
constexpr int kProbeWG = 512;
__device__ inline unsigned long long probe_clock() { return __builtin_amdgcn_s_memrealtime(); }
__device__ inline void probe_record(unsigned long long* base, int slot, unsigned long long t0) {
  const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if (wg < kProbeWG) {
    const unsigned long long t1 = probe_clock();
    *reinterpret_cast<ulonglong2*>(base + 2 * ((long)slot * kProbeWG + wg)) = make_ulonglong2(t0, t1);
  }
}

}  // namespace wmx
