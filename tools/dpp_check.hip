#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__device__ inline float sum_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
  return v;
}
__global__ void k(const float* p, float* o) { o[threadIdx.x] = sum_dpp(p[threadIdx.x]); }
int main() {
  float h[64], r[64]; double ref = 0;
  for (int i = 0; i < 64; ++i) { h[i] = (float)((i * 37) % 64) + 0.25f * i; ref += h[i]; }
  float *d, *o; hipMalloc(&d, 256); hipMalloc(&o, 256);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  hipMemcpy(r, o, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) if (r[i] != r[0] || fabs(r[i] - ref) > 1e-3) { if (bad < 4) printf("lane %d %f ref %f\n", i, r[i], ref); ++bad; }
  printf(bad ? "FAIL %d\n" : "PASS\n", bad);
  return bad != 0;
}
