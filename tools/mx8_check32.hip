// Lane map of v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 A / B and e8m0 scales (run on the GPU box), the 32-row form
// of tools/mx8_check.hip: which k each of a lane's 32 bytes carries (three candidate layouts) and which lane's
// scale byte scales (row, 32-k block) (two candidate maps).  Output C (32 x 32 f32): lane l, register r holds
// row 8 (r / 4) + 4 (l / 32) + r % 4, column l % 32.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mx8_check32.hip -o tools/mx8_check32
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

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

__global__ void mfma_k(const i32x8* a, const i32x8* b, const int* sa, const int* sb, f32x16* c) {
  const int l = threadIdx.x;
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  c[l] = acc;
}

int main() {
  uint32_t s = 777;
  std::vector<uint8_t> A(32 * 64), B(32 * 64);  // A[row][k], B[col][k]
  for (int i = 0; i < 32 * 64; ++i) {
    s = s * 1664525u + 1013904223u;
    A[i] = (uint8_t)((s >> 9) & 0x7f) | (uint8_t)((s >> 20) & 0x80);
    if (((A[i] >> 3) & 15) == 15) A[i] &= 0xf7;
    s = s * 1664525u + 1013904223u;
    B[i] = (uint8_t)((s >> 9) & 0x7f) | (uint8_t)((s >> 20) & 0x80);
    if (((B[i] >> 3) & 15) == 15) B[i] &= 0xf7;
  }
  auto kmap = [](int L, int l, int j) {
    const int g = l >> 5;
    if (L == 0) return 32 * g + j;                                   // contiguous 32
    if (L == 1) return j < 16 ? 16 * g + j : 32 + 16 * g + (j - 16);  // two 16-B halves
    return (j >> 3) * 16 + 8 * g + (j & 7);                          // 8-B interleave
  };
  int32_t *da, *db, *dsa, *dsb;
  float* dc;
  hipMalloc(&da, 64 * 32);
  hipMalloc(&db, 64 * 32);
  hipMalloc(&dsa, 64 * 4);
  hipMalloc(&dsb, 64 * 4);
  hipMalloc(&dc, 64 * 64);
  int bad = 0, found = -1;
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
          la[l * 32 + j] = A[(l & 31) * 64 + kmap(L, l, j)];
          lb[l * 32 + j] = B[(l & 31) * 64 + kmap(L, l, j)];
        }
      hipMemcpy(da, la.data(), 64 * 32, hipMemcpyHostToDevice);
      hipMemcpy(db, lb.data(), 64 * 32, hipMemcpyHostToDevice);
      hipMemcpy(dsa, sa.data(), 64 * 4, hipMemcpyHostToDevice);
      hipMemcpy(dsb, sb.data(), 64 * 4, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(mfma_k, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, dsa, dsb, (f32x16*)dc);
      std::vector<float> c(64 * 16);
      hipMemcpy(c.data(), dc, 64 * 64, hipMemcpyDeviceToHost);
      for (int S = 0; S < (pass ? 2 : 1); ++S) {
        double maxerr = 0, maxv = 0;
        for (int l = 0; l < 64; ++l)
          for (int r = 0; r < 16; ++r) {
            const int row = 8 * (r / 4) + 4 * (l / 32) + r % 4, col = l % 32;
            double ref = 0;
            for (int k = 0; k < 64; ++k) {
              const int b = k >> 5;
              const int lane_a = S == 0 ? row + 32 * b : row * 2 + b, lane_b = S == 0 ? col + 32 * b : col * 2 + b;
              const double as = std::ldexp(1.0, sa[lane_a & 63] - 127), bs = std::ldexp(1.0, sb[lane_b & 63] - 127);
              ref += (double)e4m3_decode(A[row * 64 + k]) * as * (double)e4m3_decode(B[col * 64 + k]) * bs;
            }
            maxerr = std::fmax(maxerr, std::fabs(ref - c[l * 16 + r]));
            maxv = std::fmax(maxv, std::fabs(ref));
          }
        const bool ok = maxerr <= 1e-4 * maxv + 1e-6;
        printf("pass %d layout %d scalemap %d: max |err| %.3g (max |C| %.3g) %s\n", pass, L, S, maxerr, maxv,
               ok ? "MATCH" : "");
        if (ok && pass == 0) found = L;
      }
    }
  }
  bad += found < 0;
  printf(bad ? "FAIL\n" : "PASS\n");
  return bad;
}
