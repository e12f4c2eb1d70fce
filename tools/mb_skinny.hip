// Variant sweep for the decode (skinny-M) GEMM: NW waves split K, NCT 16-column tiles per workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../realtime-whisper-asr_amd/csrc/wmx_common.h"
using namespace wmx;

template <int MT, int NW, int NCT, int KU>
__global__ __launch_bounds__(NW * 64) void sk(const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ W,
                                              int ldw, int M, int N, int K, uint16_t* __restrict__ O) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = blockIdx.x * 16 * NCT;
  const int ksteps = K / 32;
  const int per = (ksteps + NW - 1) / NW;
  const int ks0 = wave * per, ks1 = min(ksteps, ks0 + per);
  f32x4 acc[MT][NCT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  const uint16_t* wrow[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) wrow[j] = W + (long)min(n0 + j * 16 + fr, N - 1) * ldw + 8 * fq;
  const uint16_t* arow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) arow[i] = A + (long)min(i * 16 + fr, M - 1) * lda + 8 * fq;
  for (int kk = ks0; kk < ks1; kk += KU) {
    u16x8 b[KU][NCT], av[KU][MT];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int k = min(kk + u, ks1 - 1) * 32;
#pragma unroll
      for (int j = 0; j < NCT; ++j) b[u][j] = *reinterpret_cast<const u16x8*>(wrow[j] + k);
#pragma unroll
      for (int i = 0; i < MT; ++i) av[u][i] = *reinterpret_cast<const u16x8*>(arow[i] + k);
    }
#pragma unroll
    for (int u = 0; u < KU; ++u)
      if (kk + u < ks1)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NCT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, av[u][i]), __builtin_bit_cast(bf16x8, b[u][j]), acc[i][j], 0, 0, 0);
  }
  constexpr int LDR = 16 * NCT + 1;
  if (NW > 1) {
    float* mine = red + (long)wave * MT * 16 * LDR;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) mine[(i * 16 + fq * 4 + r) * LDR + j * 16 + fr] = acc[i][j][r];
    __syncthreads();
    for (int idx = tid; idx < MT * 16 * 16 * NCT; idx += NW * 64) {
      const int row = idx / (16 * NCT), col = idx % (16 * NCT);
      if (row >= M || n0 + col >= N) continue;
      float v = 0.f;
      for (int w = 0; w < NW; ++w) v += red[((long)w * MT * 16 + row) * LDR + col];
      O[(long)row * N + n0 + col] = f32_to_bf16(v);
    }
  } else {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r, col = n0 + j * 16 + fr;
          if (row < M && col < N) O[(long)row * N + col] = f32_to_bf16(acc[i][j][r]);
        }
  }
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

uint16_t *A, *W, *O;
hipStream_t st;
// rotate through 8 weight copies (> 256 MB) so weights come from HBM, not the Infinity Cache
long wstride = 0;

template <int MT, int NW, int NCT, int KU>
void run(int M, int N, int K) {
  const size_t smem = NW > 1 ? (size_t)NW * MT * 16 * (16 * NCT + 1) * 4 : 0;
  if (smem > 65536) hipFuncSetAttribute((const void*)sk<MT, NW, NCT, KU>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (smem > 160 * 1024) return;
  int it = 0;
  float us = timeit([&] {
    const uint16_t* w = W + (it++ % 8) * wstride;
    hipLaunchKernelGGL((sk<MT, NW, NCT, KU>), dim3((N + 16 * NCT - 1) / (16 * NCT)), dim3(NW * 64), smem, st, A, K, w, K, M, N, K, O);
  }, st, 64);
  printf("M=%3d N=%5d K=%4d MT=%2d NW=%2d NCT=%d KU=%d: %7.2f us %7.1f GB/s\n", M, N, K, MT, NW, NCT, KU, us, 2.0 * N * K / us / 1e3);
}

int main() {
  hipStreamCreate(&st);
  wstride = 51866L * 1280 + 4096;
  hipMalloc(&A, 256L * 5120 * 2);
  hipMalloc(&W, 8 * wstride * 2);
  hipMalloc(&O, 256L * 51866 * 2);
  hipMemset(A, 0, 256L * 5120 * 2);
  hipMemset(W, 0x11, 8 * wstride * 2);
  for (int K : {1280, 5120}) {
    const int N = K == 1280 ? 1280 : 1280;
    run<4, 4, 1, 4>(40, N, K);
    run<4, 16, 1, 4>(40, N, K);
    run<4, 16, 1, 1>(40, N, K);
    run<4, 8, 2, 2>(40, N, K);
    run<4, 16, 2, 2>(40, N, K);
    run<4, 4, 4, 2>(40, N, K);
    run<4, 8, 4, 2>(40, N, K);
    run<4, 16, 4, 1>(40, N, K);
    run<4, 1, 1, 8>(40, N, K);
    run<4, 1, 4, 4>(40, N, K);
  }
  for (int N : {5120, 51866}) {
    run<4, 4, 1, 4>(40, N, 1280);
    run<4, 16, 1, 4>(40, N, 1280);
    run<4, 4, 4, 2>(40, N, 1280);
    run<4, 8, 4, 2>(40, N, 1280);
    run<4, 1, 4, 4>(40, N, 1280);
    run<4, 2, 4, 4>(40, N, 1280);
  }
  run<12, 4, 1, 1>(160, 1280, 1280);
  run<12, 8, 1, 1>(160, 1280, 1280);
  run<12, 4, 2, 1>(160, 1280, 1280);
  run<12, 2, 4, 1>(160, 1280, 1280);
  run<12, 4, 2, 1>(160, 5120, 1280);
  run<12, 2, 4, 1>(160, 5120, 1280);
  run<12, 1, 4, 1>(160, 51866, 1280);
  run<12, 2, 4, 1>(160, 51866, 1280);
  return 0;
}
