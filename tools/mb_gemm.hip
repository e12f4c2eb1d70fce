// Microbenchmark: launch floor, HBM copy, skinny / tiled GEMM shapes of the decode step (HIP events, one process).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../realtime-whisper-asr_amd/csrc/wmx_kernels.h"
using namespace wmx;

__global__ void empty_k() {}
__global__ void copy_k(const float4* __restrict__ a, float4* __restrict__ b, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) b[i] = a[i];
}

template <class F>
static float timeit(F f, hipStream_t st, int iters = 50) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipStreamSynchronize(st);
  hipEventRecord(a, st);
  for (int i = 0; i < iters; ++i) f();
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / iters;
}

int main() {
  hipStream_t st;
  hipStreamCreate(&st);
  gemm_init_attributes();
  printf("empty kernel: %.2f us\n", timeit([&] { hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st); }, st, 200));
  printf("empty 1024 WGs: %.2f us\n", timeit([&] { hipLaunchKernelGGL(empty_k, dim3(1024), dim3(256), 0, st); }, st, 200));
  const long nbytes = 1L << 30;
  float *x, *y;
  hipMalloc(&x, nbytes);
  hipMalloc(&y, nbytes);
  hipMemset(x, 0, nbytes);
  for (long mb : {4L, 16L, 64L, 512L}) {
    long n4 = mb * (1 << 20) / 16;
    float us = timeit([&] { hipLaunchKernelGGL(copy_k, dim3(std::min<long>(n4 / 256 + 1, 8192)), dim3(256), 0, st, (float4*)x, (float4*)y, n4); }, st);
    printf("copy %4ld MB: %8.2f us  %7.1f GB/s (read+write)\n", mb, us, 2.0 * mb * (1 << 20) / us / 1e3);
  }
  uint16_t *A, *W, *O;
  float* bias;
  hipMalloc(&A, 256L * 5120 * 2);
  hipMalloc(&W, 51866L * 5120 * 2);
  hipMalloc(&O, 256L * 51866 * 4);
  hipMalloc(&bias, 51866 * 4);
  hipMemset(A, 0, 256L * 5120 * 2);
  hipMemset(W, 0, 51866L * 5120 * 2);
  hipMemset(bias, 0, 51866 * 4);
  struct Shape { int M, N, K; };
  for (Shape s : {Shape{40, 1280, 1280}, Shape{40, 3840, 1280}, Shape{40, 5120, 1280}, Shape{40, 1280, 5120},
                  Shape{40, 51866, 1280}, Shape{8, 1280, 1280}, Shape{160, 1280, 1280}, Shape{160, 5120, 1280},
                  Shape{160, 1280, 5120}, Shape{160, 51866, 1280}}) {
    for (int tile : {TILE_SKINNY, TILE_64x64}) {
      GemmCall g;
      g.A = A; g.lda = s.K; g.W = W; g.ldw = s.K; g.M = s.M; g.N = s.N; g.K = s.K;
      g.epi.kind = EPI_STORE16; g.epi.bias = bias; g.epi.out = O; g.epi.ldc = s.N;
      g.tile = tile;
      float us = timeit([&] { launch_gemm(DT::BF16, g, st); }, st);
      double wb = 2.0 * s.N * s.K;
      printf("gemm M=%3d N=%5d K=%4d %s: %8.2f us  weights %6.1f MB  %7.1f GB/s\n", s.M, s.N, s.K,
             tile == TILE_SKINNY ? "skinny" : "64x64 ", us, wb / 1e6, wb / us / 1e3);
    }
  }
  return 0;
}
