// Decode-GEMM sweep: K split across S workgroups (4 waves each split their chunk again), partial tiles written as
// f32 slabs [S][M][N], then a separate deterministic reduce kernel.  Weights rotate through 8 copies (> 1 GB) so
// every launch streams them from HBM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../realtime-whisper-asr_amd/csrc/wmx_common.h"
using namespace wmx;

// KSPLIT: the 4 waves of a workgroup split its K chunk (LDS reduce); otherwise they own 4 different column groups.
template <int MT, int NCT, int KU, bool KSPLIT, int VAR = 0>
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
  // VAR 1: fragment-major W: tile (n/16, k/32) is one contiguous 1 KiB, lane-linear
  const int ksteps_all = K / 32;
  const uint16_t* wtile[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) wtile[j] = W + ((long)min((n0 + j * 16) / 16, (N - 1) / 16) * ksteps_all) * 512 + lane * 8;
  const uint16_t* arow[MT];
  const uint16_t* Ab = VAR == 2 ? A + (long)(blockIdx.x % 64) * 64 * lda : A;
#pragma unroll
  for (int i = 0; i < MT; ++i) arow[i] = Ab + (long)min(i * 16 + fr, M - 1) * lda + 8 * fq;
  for (int kk = ks0; kk < ks1; kk += KU) {
    u16x8 b[KU][NCT], av[KU][MT];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (kk + u < ks1) {
        const int k = (kk + u) * 32;
#pragma unroll
        for (int j = 0; j < NCT; ++j)
          b[u][j] = VAR == 1 ? *reinterpret_cast<const u16x8*>(wtile[j] + (long)(kk + u) * 512)
                             : *reinterpret_cast<const u16x8*>(wrow[j] + k);
#pragma unroll
        for (int i = 0; i < MT; ++i)
          av[u][i] = VAR == 3 ? u16x8{(uint16_t)k, 1, 2, 3, 4, 5, 6, (uint16_t)i} : *reinterpret_cast<const u16x8*>(arow[i] + k);
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
  if (VAR == 4) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == 1234.5f) P[tid] = t;
    return;
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
int g_rot = 8;

template <int MT, int NCT, int KU, bool KSPLIT, int VAR = 0>
void run(int M, int N, int K, int S) {
  int it = 0;
  const int cols = KSPLIT ? 16 * NCT : 64 * NCT;
  const int tiles = (N + cols - 1) / cols;
  float us_p = timeit([&] {
    const uint16_t* w = W + (it++ % g_rot) * wstride;
    hipLaunchKernelGGL((part<MT, NCT, KU, KSPLIT, VAR>), dim3(tiles, S), dim3(256), 0, st, A, K, w, K, M, N, K, S, P);
  }, st);
  printf("rot=%d M=%3d N=%5d K=%4d MT=%2d NCT=%d KU=%d %s S=%3d WG=%6d VAR=%d: part %7.2f us (%6.0f GB/s)\n", g_rot, M, N,
         K, MT, NCT, KU, KSPLIT ? "ksplit" : "nsplit", S, tiles * S, VAR, us_p, 2.0 * N * K / us_p / 1e3);
}

int main() {
  hipStreamCreate(&st);
  wstride = 51866L * 1280 + 4096;
  hipMalloc(&A, 64L * 64 * 5120 * 2);
  hipMalloc(&W, 8 * wstride * 2);
  hipMalloc(&O, 256L * 51866 * 2);
  hipMalloc(&P, 64L * 256 * 5120 * 4);
  hipMemset(A, 0, 64L * 64 * 5120 * 2);
  hipMemset(W, 0x11, 8 * wstride * 2);
  for (int rot : {8, 1}) {
    g_rot = rot;
    run<3, 2, 2, true, 1>(40, 1280, 1280, 8);
    run<3, 2, 2, true, 1>(40, 3840, 1280, 4);
    run<3, 2, 2, true, 1>(40, 5120, 1280, 1);
    run<3, 2, 2, true, 1>(40, 5120, 1280, 4);
    run<3, 4, 2, true, 1>(40, 1280, 5120, 8);
    run<3, 4, 2, true, 1>(40, 51866, 1280, 1);
  }
  return 0;
}
