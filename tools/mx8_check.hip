// Unit check of the gfx950 MX-fp8 primitives libwmx relies on (run on the GPU box):
//  1. v_cvt_pk_fp8_f32 rounds f32 -> OCP e4m3 to nearest-even (compared with a C restatement on 2^20 values);
//  2. v_mfma_scale_f32_16x16x128_f8f6f4 (A, B e4m3, e8m0 scales): lane l (g = l >> 4) holds row (l & 15),
//     k = 16g .. 16g+15 in bytes 0..15 and k = 64 + 16g .. +15 in bytes 16..31 of A (of B^T); the scale byte of
//     lane l (opsel 0) scales row (l & 15), k-block (l >> 4) (k = 32 (l >> 4) .. +32), whichever lane holds that
//     block's data.  (Measured: of three data layouts x two scale maps only this pair reproduces the product.)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mx8_check.hip -o tools/mx8_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static float e4m3_decode(uint8_t b) {
  const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  float v;
  if (e == 15 && m == 7) return NAN;
  if (e == 0)
    v = std::ldexp((float)m / 8.0f, -6);
  else
    v = std::ldexp(1.0f + (float)m / 8.0f, e - 7);
  return s ? -v : v;
}
// nearest-even over the 254 finite codes (brute force reference)
static uint8_t e4m3_encode_ref(float x) {
  int best = 0;
  double bd = 1e30;
  for (int b = 0; b < 256; ++b) {
    const float v = e4m3_decode((uint8_t)b);
    if (std::isnan(v)) continue;
    const double d = std::fabs((double)v - (double)x);
    if (d < bd || (d == bd && ((b & 1) == 0) && ((best & 1) == 1))) {
      bd = d;
      best = b;
    }
  }
  if (e4m3_decode((uint8_t)best) == 0.0f) best = std::signbit(x) ? 0x80 : 0;
  return (uint8_t)best;
}

__global__ void cvt_k(const float* x, uint32_t* q, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (2 * i + 1 < n) q[i] = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
}

__global__ void mfma_k(const i32x8* a, const i32x8* b, const int* sa, const int* sb, f32x4* c) {
  const int l = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  c[l] = acc;
}

int main() {
  int bad = 0;
  // ---- 1. conversion ----
  const int n = 1 << 16;
  std::vector<float> x(n);
  uint32_t s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float u = (float)(s >> 8) / 16777216.0f;  // [0,1)
    s = s * 1664525u + 1013904223u;
    const int ex = (int)(s >> 27) - 12;               // 2^-12 .. 2^19
    float v = std::ldexp(1.0f + u, ex);
    if (v > 448.f) v = 448.f * u;
    x[i] = (s & 1) ? -v : v;
  }
  float* dx;
  uint32_t* dq;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dq, n * 2);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(cvt_k, dim3(n / 512), dim3(256), 0, 0, dx, dq, n);
  std::vector<uint32_t> q(n / 2);
  hipMemcpy(q.data(), dq, n * 2, hipMemcpyDeviceToHost);
  int mism = 0;
  for (int i = 0; i < n; ++i) {
    const uint8_t got = (uint8_t)((q[i / 2] >> (8 * (i & 1))) & 0xff);
    const uint8_t ref = e4m3_encode_ref(x[i]);
    if (got != ref) {
      if (mism < 5) printf("cvt mismatch x=%.9g got 0x%02x (%g) ref 0x%02x (%g)\n", x[i], got, e4m3_decode(got), ref,
                           e4m3_decode(ref));
      ++mism;
    }
  }
  printf("cvt_pk_fp8_f32: %d / %d mismatches vs nearest-even e4m3\n", mism, n);
  bad += mism != 0;

  // ---- 2. scaled MFMA lane map: data layouts x scale mappings, first with unit scales ----
  std::vector<uint8_t> A(16 * 128), B(16 * 128);  // A[row][k], B[col][k]
  for (int i = 0; i < 16 * 128; ++i) {
    s = s * 1664525u + 1013904223u;
    A[i] = (uint8_t)((s >> 9) & 0x7f) | (uint8_t)((s >> 20) & 0x80);
    if (((A[i] >> 3) & 15) == 15) A[i] &= 0xf7;
    s = s * 1664525u + 1013904223u;
    B[i] = (uint8_t)((s >> 9) & 0x7f) | (uint8_t)((s >> 20) & 0x80);
    if (((B[i] >> 3) & 15) == 15) B[i] &= 0xf7;
  }
  // layout L: element j (0..31) of lane l -> k
  auto kmap = [](int L, int l, int j) {
    const int g = l >> 4;
    if (L == 0) return 32 * g + j;
    if (L == 1) return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);
    return (j >> 3) * 32 + 8 * g + (j & 7);
  };
  int32_t *da, *db, *dsa, *dsb;
  float* dc;
  hipMalloc(&da, 64 * 32);
  hipMalloc(&db, 64 * 32);
  hipMalloc(&dsa, 64 * 4);
  hipMalloc(&dsb, 64 * 4);
  hipMalloc(&dc, 64 * 16);
  int found = -1;
  for (int pass = 0; pass < 2; ++pass) {
    std::vector<int> sa(64, 127), sb(64, 127);
    if (pass == 1)
      for (int l = 0; l < 64; ++l) {
        s = s * 1664525u + 1013904223u;
        sa[l] = 127 + (int)((s >> 10) % 9) - 4;
        s = s * 1664525u + 1013904223u;
        sb[l] = 127 + (int)((s >> 10) % 9) - 4;
      }
    for (int L = 0; L < 3; ++L) {
      std::vector<uint8_t> la(64 * 32), lb(64 * 32);
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
          la[l * 32 + j] = A[(l & 15) * 128 + kmap(L, l, j)];
          lb[l * 32 + j] = B[(l & 15) * 128 + kmap(L, l, j)];
        }
      hipMemcpy(da, la.data(), 64 * 32, hipMemcpyHostToDevice);
      hipMemcpy(db, lb.data(), 64 * 32, hipMemcpyHostToDevice);
      hipMemcpy(dsa, sa.data(), 64 * 4, hipMemcpyHostToDevice);
      hipMemcpy(dsb, sb.data(), 64 * 4, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(mfma_k, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, dsa, dsb, (f32x4*)dc);
      std::vector<float> c(64 * 4);
      hipMemcpy(c.data(), dc, 64 * 16, hipMemcpyDeviceToHost);
      // scale map S: scale of (row r, 32-block b) comes from lane S(r, b)
      for (int S = 0; S < (pass ? 2 : 1); ++S) {
        double maxerr = 0, maxv = 0;
        for (int l = 0; l < 64; ++l)
          for (int r = 0; r < 4; ++r) {
            const int row = (l >> 4) * 4 + r, col = l & 15;
            double ref = 0;
            for (int k = 0; k < 128; ++k) {
              const int b = k >> 5;
              const int lane_a = S == 0 ? row + 16 * b : row * 4 + b, lane_b = S == 0 ? col + 16 * b : col * 4 + b;
              const double as = std::ldexp(1.0, sa[lane_a & 63] - 127), bs = std::ldexp(1.0, sb[lane_b & 63] - 127);
              ref += (double)e4m3_decode(A[row * 128 + k]) * as * (double)e4m3_decode(B[col * 128 + k]) * bs;
            }
            maxerr = std::fmax(maxerr, std::fabs(ref - c[l * 4 + r]));
            maxv = std::fmax(maxv, std::fabs(ref));
          }
        const bool ok = maxerr <= 1e-4 * maxv + 1e-6;  // f32 accumulation inside the MFMA
        printf("pass %d layout %d scalemap %d: max |err| %.3g (max |C| %.3g) %s\n", pass, L, S, maxerr, maxv,
               ok ? "MATCH" : "");
        if (ok && pass == 0) found = L;
        if (pass == 1 && S == 0 && L == 1) bad += !ok;  // the layout and scale map libwmx uses
      }
    }
  }
  bad += found < 0;
  printf(bad ? "FAIL\n" : "PASS\n");
  return bad;
}
