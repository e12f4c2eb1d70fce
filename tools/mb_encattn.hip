// Microbenchmark: encoder self-attention (B windows x H heads x 1500 x 64), the 16x16 flash kernel vs the
// 32x32 enc_attn kernel; checks the two against each other on random bf16 q/k/v and prints TFLOP/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_encattn.hip -o tools/mb_encattn
#include "../realtime-whisper-asr_amd/csrc/wmx_attn.hip"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace wmx;

__global__ void fill_k(uint16_t* p, long n, uint32_t seed, float scale) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    uint32_t z = (uint32_t)i * 2654435761u ^ seed;
    z ^= z >> 15;
    z *= 2246822519u;
    z ^= z >> 13;
    const float u = ((float)(z >> 8) * (1.0f / 8388608.0f) - 1.0f) * scale;
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
  const int B = argc > 1 ? atoi(argv[1]) : 8, H = 20, T = 1500, d = H * 64;
  const float qscale = argc > 2 ? atof(argv[2]) : 4.0f;
  const long n = (long)B * T * 3 * d;
  uint16_t *qkv, *o1, *o2;
  hipMalloc(&qkv, n * 2);
  hipMalloc(&o1, (long)B * T * d * 2);
  hipMalloc(&o2, (long)B * T * d * 2);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, qkv, n, 3u, qscale);
  AttnArgs a{};
  a.q = qkv;
  a.k = qkv + d;
  a.v = qkv + 2 * d;
  a.q_ld = a.k_ld = a.v_ld = 3 * d;
  a.q_bstride = a.k_bstride = a.v_bstride = (long)T * 3 * d;
  a.o = o1;
  a.o_ld = d;
  a.o_bstride = (long)T * d;
  a.B = B;
  a.H = H;
  a.Tq = a.Tk = T;
  a.head_stride = 64;
  const double fl = 4.0 * B * H * (double)T * T * 64;
  const float t1 = timeit([&] { launch_attn_flash(DT::BF16, a, 0, 0, nullptr, 0); }, 20);
  AttnArgs a2 = a;
  a2.o = o2;
  const float t2 = timeit([&] { launch_attn_encoder(DT::BF16, a2, 0); }, 20);
  hipDeviceSynchronize();
  const long no = (long)B * T * d;
  std::vector<uint16_t> x(no), y(no);
  hipMemcpy(x.data(), o1, no * 2, hipMemcpyDeviceToHost);
  hipMemcpy(y.data(), o2, no * 2, hipMemcpyDeviceToHost);
  double maxd = 0, maxv = 0, se = 0, sx = 0;
  for (long i = 0; i < no; ++i) {
    const double u = bf16_to_f32(x[i]), v = bf16_to_f32(y[i]);
    maxd = std::fmax(maxd, std::fabs(u - v));
    maxv = std::fmax(maxv, std::fabs(u));
    se += (u - v) * (u - v);
    sx += u * u;
  }
  const double rel = std::sqrt(se / std::fmax(sx, 1e-30));
  const bool ok = rel < 1e-2;
  printf("enc attn B=%d H=%d T=%d: flash16 %8.1f us %6.1f TF/s | enc32 %8.1f us %6.1f TF/s  x%.2f  maxdiff %.3g/%.3g relL2 %.3g %s\n",
         B, H, T, t1 * 1e3, fl / t1 / 1e9, t2 * 1e3, fl / t2 / 1e9, t1 / t2, maxd, maxv, rel, ok ? "ok" : "MISMATCH");
  return ok ? 0 : 1;
}
