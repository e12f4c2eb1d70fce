// Decode-GEMM sweep: K split across S workgroups (4 waves each split their chunk again), partial tiles written as
// f32 slabs [S][M][N], then a separate deterministic reduce kernel.  Weights rotate through 8 copies (> 1 GB) so
// every launch streams them from HBM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../realtime-whisper-asr_amd/csrc/wmx_common.h"
using namespace wmx;

// KSPLIT: the 4 waves of a workgroup split its K chunk (LDS reduce); otherwise they own 4 different column groups.
template <int MT, int NCT, int KU, bool KSPLIT>
__global__ __launch_bounds__(256) void part(const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ W,
                                            int ldw, int M, int N, int K, int S, float* __restrict__ P) {
  __shared__ float red[KSPLIT ? 4 : 1][KSPLIT ? MT * 16 : 1][KSPLIT ? 16 * NCT + 1 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = KSPLIT ? blockIdx.x * 16 * NCT : (blockIdx.x * 4 + wave) * 16 * NCT;
  const int sp = blockIdx.y;
  const int ksteps = K / 32, kps = (ksteps + S - 1) / S;
  const int kb = sp * kps, ke = min(ksteps, kb + kps);
  int ks0 = kb, ks1 = ke;
  if (KSPLIT) {
    const int per = (max(0, ke - kb) + 3) / 4;
    ks0 = kb + wave * per;
    ks1 = min(ke, ks0 + per);
  }
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
      if (kk + u < ks1) {
        const int k = (kk + u) * 32;
#pragma unroll
        for (int j = 0; j < NCT; ++j) b[u][j] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wrow[j] + k));
#pragma unroll
        for (int i = 0; i < MT; ++i) av[u][i] = *reinterpret_cast<const u16x8*>(arow[i] + k);
      }
    }
#pragma unroll
    for (int u = 0; u < KU; ++u)
      if (kk + u < ks1)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NCT; ++j) acc[i][j] = mfma16<DT::BF16>(av[u][i], b[u][j], acc[i][j]);
  }
  if (KSPLIT) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave][i * 16 + fq * 4 + r][j * 16 + fr] = acc[i][j][r];
    __syncthreads();
    for (int idx = tid; idx < MT * 16 * 16 * NCT; idx += 256) {
      const int row = idx / (16 * NCT), col = idx % (16 * NCT);
      if (row < M && n0 + col < N)
        P[((long)sp * M + row) * N + n0 + col] =
            red[0][row][col] + red[1][row][col] + red[2][row][col] + red[3][row][col];
    }
  } else {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r, col = n0 + j * 16 + fr;
          if (row < M && col < N) P[((long)sp * M + row) * N + col] = acc[i][j][r];
        }
  }
}

__global__ __launch_bounds__(256) void reduce(const float* __restrict__ P, int S, int M, int N, uint16_t* __restrict__ O) {
  const long i4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= (long)M * N) return;
  float4 a = make_float4(0, 0, 0, 0);
  for (int s = 0; s < S; ++s) {
    const float4 x = *reinterpret_cast<const float4*>(P + (long)s * M * N + i4);
    a.x += x.x;
    a.y += x.y;
    a.z += x.z;
    a.w += x.w;
  }
  O[i4] = f32_to_bf16(a.x);
  O[i4 + 1] = f32_to_bf16(a.y);
  O[i4 + 2] = f32_to_bf16(a.z);
  O[i4 + 3] = f32_to_bf16(a.w);
}

template <class F>
static float timeit(F f, hipStream_t st, int iters = 64) {
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
float* P;
hipStream_t st;
long wstride = 0;

template <int MT, int NCT, int KU, bool KSPLIT>
void run(int M, int N, int K, int S) {
  int it = 0;
  const int cols = KSPLIT ? 16 * NCT : 64 * NCT;
  const int tiles = (N + cols - 1) / cols;
  float us_p = timeit([&] {
    const uint16_t* w = W + (it++ % 8) * wstride;
    hipLaunchKernelGGL((part<MT, NCT, KU, KSPLIT>), dim3(tiles, S), dim3(256), 0, st, A, K, w, K, M, N, K, S, P);
  }, st);
  const int rb = (int)(((long)M * N / 4 + 255) / 256);
  float us_r = timeit([&] { hipLaunchKernelGGL(reduce, dim3(rb), dim3(256), 0, st, P, S, M, N, O); }, st);
  printf("M=%3d N=%5d K=%4d MT=%2d NCT=%d KU=%d %s S=%3d WG=%6d: part %7.2f us (%6.0f GB/s) reduce %6.2f us\n", M,
         N, K, MT, NCT, KU, KSPLIT ? "ksplit" : "nsplit", S, tiles * S, us_p, 2.0 * N * K / us_p / 1e3, us_r);
}

int main() {
  hipStreamCreate(&st);
  wstride = 51866L * 1280 + 4096;
  hipMalloc(&A, 256L * 5120 * 2);
  hipMalloc(&W, 8 * wstride * 2);
  hipMalloc(&O, 256L * 51866 * 2);
  hipMalloc(&P, 64L * 256 * 5120 * 4);
  hipMemset(A, 0, 256L * 5120 * 2);
  hipMemset(W, 0x11, 8 * wstride * 2);
  const int shapes[5][2] = {{1280, 1280}, {3840, 1280}, {5120, 1280}, {1280, 5120}, {51866, 1280}};
  for (auto& sh : shapes) {
    const int N = sh[0], K = sh[1];
    for (int S : {1, 2, 4, 8, 10, 20}) {
      if (K / 32 < S * 2) continue;
      if ((long)S * 40 * N > 64L * 256 * 5120) continue;
      if (N > 6000 && S > 2) continue;
      run<3, 1, 2, true>(40, N, K, S);
      run<3, 2, 2, true>(40, N, K, S);
      run<3, 4, 2, true>(40, N, K, S);
      run<3, 1, 4, false>(40, N, K, S);
      run<3, 2, 4, false>(40, N, K, S);
      run<3, 4, 2, false>(40, N, K, S);
    }
  }
  for (int S : {1, 4, 10}) run<10, 2, 1, false>(160, 1280, 1280, S);
  for (int S : {1, 4, 10}) run<10, 2, 1, false>(160, 1280, 5120, S * 2);
  for (int S : {1, 4, 10}) run<10, 1, 1, true>(160, 1280, 5120, S * 2);
  for (int S : {1, 2}) run<10, 2, 1, false>(160, 51866, 1280, S);
  for (int S : {1, 2}) run<10, 4, 1, false>(160, 51866, 1280, S);
  return 0;
}
