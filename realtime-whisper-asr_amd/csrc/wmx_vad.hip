// Silero VAD v5, 16 kHz branch, batched over streams (the reference calls the torch.hub model
// once per 512-sample window, asr_components.py:96 and :58-78).  Two launches per call:
//
//  * vad_encode_kernel: one 16-wave workgroup per (stream, window) -- every window's context-free part at once.  The
//    576-sample input (64 context samples + 512 new ones; the context of a stream's first window comes from its
//    slot, of later windows from the same call's audio) and its right reflection pad land in LDS; the STFT-as-conv
//    (258 basis rows x 256 taps x 4 frames) runs one wave per basis row with lanes over taps, so every basis load
//    is a coalesced 256-byte row piece and each (row, frame) dot product ends in a DPP wave sum; the magnitudes
//    [129][4] and the four conv + ReLU layers (129->128 s1, 128->64 s2, 64->64 s2, 64->128 s1) stay in LDS, one
//    wave per output channel with lanes over (input channel, tap).  Output: the [128] encoder vector per window.
//  * vad_decode_kernel: one workgroup per stream, its windows in order (the LSTM recursion is the only sequential
//    part): thread j computes gate j from the transposed W_ih^T / W_hh^T images ([128][512], so the 512 threads
//    read one contiguous 2 KiB row per k), then the cell update, ReLU -> 1x1 conv -> sigmoid as a wave sum.  The
//    slot's (h, c) and 64-sample context are written back at the end.
//
// f32 throughout (the oracle, oracle/silero_np.py, is float64; tolerance in tests/test_gpu_vad.py).  This is
// latency-bound work of ~0.55 MFLOP per window on L2-resident weights (1.2 MB): no MFMA.
#include "wmx_common.h"
#include "wmx_kernels.h"

namespace wmx {

namespace {

__device__ inline float vad_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

// one conv1d(kernel 3, padding 1) + ReLU layer over LDS images in[CIN][LIN] -> out[COUT][LOUT]; one wave per output
// channel, lanes over the CIN * 3 (channel, tap) products (contiguous weight reads)
template <int CIN, int COUT, int LIN, int STRIDE>
__device__ inline void vad_conv(const float* __restrict__ w, const float* __restrict__ b, const float* in,
                                float* out, int wave, int lane, int nwaves) {
  constexpr int LOUT = (LIN - 1) / STRIDE + 1;
  for (int o = wave; o < COUT; o += nwaves) {
    float acc[LOUT];
#pragma unroll
    for (int t = 0; t < LOUT; ++t) acc[t] = 0.f;
    for (int j = lane; j < CIN * 3; j += 64) {
      const int i = j / 3, k = j - 3 * i;
      const float wv = w[(long)o * CIN * 3 + j];
#pragma unroll
      for (int t = 0; t < LOUT; ++t) {
        const int p = t * STRIDE + k - 1;
        if (p >= 0 && p < LIN) acc[t] = fmaf(wv, in[i * LIN + p], acc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < LOUT; ++t) acc[t] = wave_sum(acc[t]);
    if (lane == 0) {
#pragma unroll
      for (int t = 0; t < LOUT; ++t) out[o * LOUT + t] = fmaxf(acc[t] + b[o], 0.f);
    }
  }
}

}  // namespace

constexpr int kVadEncThreads = 1024;  // 16 waves: each layer's channels split 16 ways (the per-window chain is
                                      // latency-bound: wave sums and dependent weight loads per channel)

__global__ __launch_bounds__(kVadEncThreads) void vad_encode_kernel(const float* __restrict__ W, const float* __restrict__ pcm,
                                                         long stride, const float* __restrict__ ctx,
                                                         const int* __restrict__ slots, int nwin,
                                                         float* __restrict__ enc) {
  const int n = blockIdx.x, s = n / nwin, wi = n - s * nwin;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kVadEncThreads / 64;
  __shared__ float xs[kVadPadded];
  __shared__ float mag[129 * 4];
  __shared__ float h1[128 * 4], h2[64 * 2], h3[64];
  const float* src = pcm + (long)s * stride;
  const float* cx = ctx + (long)slots[s] * kVadContext;
  for (int i = tid; i < kVadInput; i += kVadEncThreads) {
    const long idx = (long)wi * kVadWindow - kVadContext + i;
    xs[i] = idx >= 0 ? src[idx] : cx[idx + kVadContext];
  }
  __syncthreads();
  // ReflectionPad1d((0, 64)): xs[576 + i] = xs[574 - i]
  if (tid < kVadPadded - kVadInput) xs[kVadInput + tid] = xs[kVadInput - 2 - tid];
  __syncthreads();

  // STFT magnitudes: wave per frequency bin c (real row c, imaginary row 129 + c), lanes over the 256 taps
  const float* basis = W + kVadOffBasis;
  for (int c = wave; c < 129; c += NW) {
    float re[4] = {0.f, 0.f, 0.f, 0.f}, im[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = lane + 64 * j;
      const float br = basis[c * 256 + k], bi = basis[(129 + c) * 256 + k];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        re[t] = fmaf(br, xs[t * 128 + k], re[t]);
        im[t] = fmaf(bi, xs[t * 128 + k], im[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float r = wave_sum(re[t]), q = wave_sum(im[t]);
      if (lane == 0) mag[c * 4 + t] = sqrtf(r * r + q * q);
    }
  }
  __syncthreads();
  vad_conv<129, 128, 4, 1>(W + kVadOffC0w, W + kVadOffC0b, mag, h1, wave, lane, NW);
  __syncthreads();
  vad_conv<128, 64, 4, 2>(W + kVadOffC1w, W + kVadOffC1b, h1, h2, wave, lane, NW);
  __syncthreads();
  vad_conv<64, 64, 2, 2>(W + kVadOffC2w, W + kVadOffC2b, h2, h3, wave, lane, NW);
  __syncthreads();
  vad_conv<64, 128, 1, 1>(W + kVadOffC3w, W + kVadOffC3b, h3, enc + (long)n * kVadHidden, wave, lane, NW);
}

__global__ __launch_bounds__(512) void vad_decode_kernel(const float* __restrict__ W, const float* __restrict__ enc,
                                                         int nwin, const int* __restrict__ slots,
                                                         float* __restrict__ state, float* __restrict__ ctx,
                                                         const float* __restrict__ pcm, long stride,
                                                         float* __restrict__ probs) {
  const int s = blockIdx.x, slot = slots[s];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float x[kVadHidden], h[kVadHidden], c[kVadHidden], g[4 * kVadHidden];
  float* st = state + (long)slot * 2 * kVadHidden;
  if (tid < kVadHidden) {
    h[tid] = st[tid];
    c[tid] = st[kVadHidden + tid];
  }
  const float* wihT = W + kVadOffWihT;  // [128][512]
  const float* whhT = W + kVadOffWhhT;  // [128][512]
  const float bias = W[kVadOffBih + tid] + W[kVadOffBhh + tid];
  for (int wi = 0; wi < nwin; ++wi) {
    if (tid < kVadHidden) x[tid] = enc[((long)s * nwin + wi) * kVadHidden + tid];
    __syncthreads();
    // gate tid: two independent chains per matrix keep more loads in flight
    float a0 = 0.f, a1 = 0.f, b0 = 0.f, b1 = 0.f;
#pragma unroll 8
    for (int k = 0; k < kVadHidden; k += 2) {
      a0 = fmaf(wihT[k * 512 + tid], x[k], a0);
      a1 = fmaf(wihT[(k + 1) * 512 + tid], x[k + 1], a1);
      b0 = fmaf(whhT[k * 512 + tid], h[k], b0);
      b1 = fmaf(whhT[(k + 1) * 512 + tid], h[k + 1], b1);
    }
    g[tid] = (a0 + a1) + (b0 + b1) + bias;
    __syncthreads();
    if (tid < kVadHidden) {
      const float ig = vad_sigmoid(g[tid]), fg = vad_sigmoid(g[kVadHidden + tid]);
      const float gg = tanhf(g[2 * kVadHidden + tid]), og = vad_sigmoid(g[3 * kVadHidden + tid]);
      const float cn = fg * c[tid] + ig * gg;
      c[tid] = cn;
      h[tid] = og * tanhf(cn);
    }
    __syncthreads();
    if (wave == 0) {
      const float v = W[kVadOffW2 + lane] * fmaxf(h[lane], 0.f) + W[kVadOffW2 + 64 + lane] * fmaxf(h[64 + lane], 0.f);
      const float tot = wave_sum(v);
      if (lane == 0) probs[(long)s * nwin + wi] = vad_sigmoid(tot + W[kVadOffB2]);
    }
  }
  __syncthreads();
  if (tid < kVadHidden) {
    st[tid] = h[tid];
    st[kVadHidden + tid] = c[tid];
  }
  // the next call's context: the last 64 samples of this call's audio
  if (tid < kVadContext) ctx[(long)slot * kVadContext + tid] = pcm[(long)s * stride + (long)nwin * kVadWindow - kVadContext + tid];
}

void launch_vad(const float* W, const float* pcm, long stride, float* ctx, float* state, const int* slots_dev, int S,
                int nwin, float* enc, float* probs, hipStream_t st) {
  hipLaunchKernelGGL(vad_encode_kernel, dim3(S * nwin), dim3(kVadEncThreads), 0, st, W, pcm, stride, ctx, slots_dev, nwin, enc);
  hipLaunchKernelGGL(vad_decode_kernel, dim3(S), dim3(512), 0, st, W, enc, nwin, slots_dev, state, ctx, pcm, stride,
                     probs);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
