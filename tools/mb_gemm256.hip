// Microbenchmark: encoder-shape GEMMs, 128x128 two-barrier tile vs the 256x256 counted-vmcnt ring (HIP events).
// Checks the 256 tile against the 128 tile on random bf16 operands and prints TFLOP/s per shape.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_gemm256.hip -o tools/mb_gemm256
#include "../realtime-whisper-asr_amd/csrc/wmx_gemm.hip"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace wmx;

__global__ void fill_k(uint16_t* p, long n, uint32_t seed) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    uint32_t z = (uint32_t)i * 2654435761u ^ seed;
    z ^= z >> 15;
    z *= 2246822519u;
    z ^= z >> 13;
    const float u = (float)(z >> 8) * (1.0f / 8388608.0f) - 1.0f;
    p[i] = f32_to_bf16(u);
  }
}

template <class F>
static float timeit(F f, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main(int argc, char** argv) {
  gemm_init_attributes();
  struct Shape {
    const char* name;
    int M, N, K;
  } shapes[] = {{"qkv", 12000, 3840, 1280},  {"out", 12000, 1280, 1280},  {"fc1", 12000, 5120, 1280},
                {"fc2", 12000, 1280, 5120},  {"conv1", 24000, 1280, 384}, {"conv2", 12000, 1280, 3840},
                {"xkv", 12000, 81920, 1280}, {"sq4k", 4096, 4096, 4096}};
  const long maxA = 24000L * 5120, maxW = 81920L * 1280, maxC = 12000L * 81920;
  uint16_t *A, *W, *C1, *C2;
  float* bias;
  hipMalloc(&bias, 81920 * 4);
  {
    std::vector<float> hb(81920);
    for (int i = 0; i < 81920; ++i) hb[i] = 0.01f * (i % 97) - 0.4f;
    hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  }
  hipMalloc(&A, maxA * 2);
  hipMalloc(&W, maxW * 2);
  hipMalloc(&C1, maxC * 2);
  hipMalloc(&C2, maxC * 2);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, A, maxA, 1u);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, W, maxW, 7u);
  // fp8 operands: reuse the bf16 bit patterns with bit 6 cleared (never the e4m3 NaN code 0x7f / 0xff)
  uint16_t *A8, *W8;
  uint8_t* S8;
  hipMalloc(&A8, maxA);
  hipMalloc(&W8, maxW);
  hipMalloc(&S8, maxA / 32 + 4096);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, A8, maxA / 2, 3u);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, W8, maxW / 2, 5u);
  hipMemset(S8, 127, maxA / 32 + 4096);
  hipMemset(A8, 0x35, maxA);
  hipMemset(W8, 0x33, maxW);
  hipDeviceSynchronize();
  int bad = 0;
  for (const auto& s : shapes) {
    GemmCall g;
    g.A = A;
    g.lda = s.K;
    g.W = W;
    g.ldw = s.K;
    g.M = s.M;
    g.N = s.N;
    g.K = s.K;
    g.epi.kind = (argc > 1 || s.N != 5120) ? EPI_STORE16 : EPI_GELU16;
    g.epi.bias = bias;
    g.epi.ldc = s.N;
    g.epi.out = C1;
    g.tile = TILE_128x128;
    const double fl = 2.0 * s.M * s.N * s.K;
    const int iters = fl > 1e12 ? 5 : 20;
    const float t1 = timeit([&] { launch_gemm(DT::BF16, g, 0); }, iters);
    GemmCall h = g;
    h.tile = TILE_256;
    h.epi.out = C2;
    const float t2 = timeit([&] { launch_gemm(DT::BF16, h, 0); }, iters);
#ifdef WMX_G256_STAMPS
    {  // per-tile phase clocks of the last timed launch: main loop (incl. prologue) vs epilogue, in shader clocks
      static unsigned long long stv[kG256Stamps][5];
      hipMemcpyFromSymbol(stv, HIP_SYMBOL(g256_stamps), sizeof(stv));
      const int nt = std::min(kG256Stamps, ((s.M + 255) / 256) * ((s.N + 255) / 256));
      double mainc = 0, epic = 0, clk = 0;
      unsigned long long rmin = ~0ull, rmax = 0;
      for (int t = 0; t < nt; ++t) {
        mainc += (double)(stv[t][1] - stv[t][0]);
        epic += (double)(stv[t][2] - stv[t][1]);
        clk += (double)(stv[t][2] - stv[t][0]) / (double)std::max(1ull, stv[t][4] - stv[t][3]) * 0.1;  // GHz
        rmin = std::min(rmin, stv[t][3]);
        rmax = std::max(rmax, stv[t][4]);
      }
      printf("  stamps %s: main %.0f clk, epilogue %.0f clk per tile (%d tiles), in-kernel clock %.3f GHz, "
             "first tile start to last tile end %.1f us\n",
             s.name, mainc / nt, epic / nt, nt, clk / nt, (rmax - rmin) * 0.01);
    }
#endif
    hipDeviceSynchronize();
    const long n = (long)s.M * s.N;
    std::vector<uint16_t> a(n), b(n);
    hipMemcpy(a.data(), C1, n * 2, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), C2, n * 2, hipMemcpyDeviceToHost);
    double maxd = 0, maxv = 0;
    for (long i = 0; i < n; ++i) {
      const double x = bf16_to_f32(a[i]), y = bf16_to_f32(b[i]);
      maxd = std::fmax(maxd, std::fabs(x - y));
      maxv = std::fmax(maxv, std::fabs(x));
    }
    const bool ok = maxd <= 0.02 * maxv + 1e-3;
    // MX-fp8 GEMM on the same shape (random e4m3 bytes with the NaN code cleared, unit scales): timing only
    float t3 = 0.f;
    if (s.K % 128 == 0 && s.N <= 5120) {
      Mx8Call x;
      x.A = reinterpret_cast<const uint8_t*>(A8);
      x.lda = s.K;
      x.AS = S8;
      x.ldas = s.K / 32;
      x.W = reinterpret_cast<const uint8_t*>(W8);
      x.ldw = s.K;
      x.WS = S8;
      x.ldws = s.K / 32;
      x.M = s.M;
      x.N = s.N;
      x.K = s.K;
      x.epi = h.epi;  // writes C2 after the bf16 comparison above
      x.epi.kind = EPI_STORE16;
      t3 = timeit([&] { launch_gemm_mx8(DT::BF16, x, 0); }, iters);
    }

    bad += !ok;
    printf("%-6s M=%5d N=%5d K=%5d  128x128 %8.1f us %7.1f TF/s | 256x256 %8.1f us %7.1f TF/s  x%.2f  maxdiff %.3g/%.3g %s"
           " | mx8 %8.1f us %7.1f TF/s\n",
           s.name, s.M, s.N, s.K, t1 * 1e3, fl / t1 / 1e9, t2 * 1e3, fl / t2 / 1e9, t1 / t2, maxd, maxv,
           ok ? "ok" : "MISMATCH", t3 * 1e3, t3 > 0 ? fl / t3 / 1e9 : 0.0);
  }
  printf(bad ? "FAIL\n" : "PASS\n");
  return bad ? 1 : 0;
}
