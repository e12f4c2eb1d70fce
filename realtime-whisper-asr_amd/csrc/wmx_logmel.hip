// Batched log-mel front end (faster-whisper 1.2.1 FeatureExtractor semantics).
//
//   x' = pcm[0..N) ++ zeros(160); frame f covers x'[160f-200, 160f+200) with numpy 'reflect' padding;
//   periodic Hann 400; |rfft|^2 (201 bins); slaney mel; log10(max(.,1e-10)); drop the last STFT frame
//   (F = N//160 + 1 frames); per-window max-8 clamp; (x+4)/4; encoder window = frames [seek, seek+3000)
//   of the first min(3000, F-1-seek) content frames, zero padded (pad_or_trim).
//
// Kernel 1, GEMM form (logmel_raw, opt-in WMX_LOGMEL_GEMM=1; the FFT form below is the default): one workgroup = 64 consecutive frames of one window, 4 waves x 16 frames.
//   The windowed real DFT is a [frames x 400] x [400 x 416] f32 GEMM on v_mfma_f32_16x16x4_f32 (exact
//   fp32 FMA chains; bf16 would miss the 1e-4 gate).  Audio for the 64 frames (10480 samples, reflect
//   applied) is staged once in LDS; the Hann-folded cos/sin basis streams through LDS in 16-sample
//   K-chunks.  Re/Im tiles of one bin block share a lane layout, so |X|^2 is formed in registers,
//   written to LDS, reduced through the sparse slaney filterbank, log10'd, stored, and the block max
//   is folded into a per-window atomicMax.
// Kernel 2 (logmel_finalize): clamp, scale, slice [seek, seek+3000) and zero-pad.  HBM-bound.
#include "wmx_common.h"
#include "wmx_kernels.h"

namespace wmx {

constexpr int kFFT = 400, kHop = 160, kBins = 201, kBinTiles = 13, kCols = 2 * kBinTiles * 16;  // 416
constexpr int kFramesPerWG = 64, kKChunk = 16;
constexpr int kSeg = kHop * (kFramesPerWG - 1) + kFFT;  // 10480 samples

__device__ inline int enc_max(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ inline float dec_max(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

// mel filter table: per mel m: first bin, count, offset into weights
struct MelTable {
  const int* first;
  const int* count;
  const int* offset;
  const float* w;
};

__global__ __launch_bounds__(256) void logmel_raw_kernel(const float* __restrict__ pcm, long stride,
                                                         const long* __restrict__ lens, const float* __restrict__ basis,
                                                         MelTable mt, int n_mels, float* __restrict__ raw,
                                                         int fcap, int* __restrict__ wmax) {
  const int b = blockIdx.y;
  const long N = lens[b];
  const int F = (int)(N / kHop) + 1;
  const int f0 = blockIdx.x * kFramesPerWG;
  if (f0 >= F) return;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* aud = smem;                        // [kSeg]
  float* bas = smem + kSeg;                 // [2][kKChunk][kCols]   (reused as power [64][208] after the loop)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* x = pcm + (long)b * stride;
  const long Lp = N + kHop;                 // padded length
  const long period = 2 * (Lp - 1);
  const long j0 = (long)f0 * kHop - kFFT / 2;
  for (int i = tid; i < kSeg; i += 256) {
    long j = j0 + i;
    long m = j % period;
    if (m < 0) m += period;
    if (m >= Lp) m = period - m;
    aud[i] = (m < N) ? x[m] : 0.0f;
  }
  auto stage = [&](int chunk, int buf) {
    const float4* src = reinterpret_cast<const float4*>(basis + (long)chunk * kKChunk * kCols);
    float4* dst = reinterpret_cast<float4*>(bas + buf * kKChunk * kCols);
    for (int i = tid; i < kKChunk * kCols / 4; i += 256) dst[i] = src[i];
  };
  stage(0, 0);
  __syncthreads();

  f32x4 re[kBinTiles], im[kBinTiles];
#pragma unroll
  for (int t = 0; t < kBinTiles; ++t) {
    re[t] = f32x4{0, 0, 0, 0};
    im[t] = f32x4{0, 0, 0, 0};
  }
  const int arow = (wave * 16 + (lane & 15)) * kHop;  // this lane's frame start in aud[]
  const int kq = lane >> 4;
  constexpr int nchunks = kFFT / kKChunk;  // 25
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunks) stage(c + 1, buf ^ 1);
    const float* bc = bas + buf * kKChunk * kCols;
#pragma unroll
    for (int ks = 0; ks < kKChunk / 4; ++ks) {
      const int k = ks * 4 + kq;
      const float a = aud[arow + c * kKChunk + k];
      const float* brow = bc + k * kCols + (lane & 15);
#pragma unroll
      for (int t = 0; t < kBinTiles; ++t) {
        re[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, brow[t * 16], re[t], 0, 0, 0);
        im[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, brow[(kBinTiles + t) * 16], im[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // power -> LDS [64 frames][208 bins]
  float* pw = bas;
  constexpr int kPB = kBinTiles * 16;
#pragma unroll
  for (int t = 0; t < kBinTiles; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int fr = wave * 16 + (lane >> 4) * 4 + r;
      pw[fr * kPB + t * 16 + (lane & 15)] = re[t][r] * re[t][r] + im[t][r] * im[t][r];
    }
  }
  __syncthreads();
  // sparse filterbank + log10; thread -> (frame = tid & 63, mel stride 4)
  float bmax = -INFINITY;
  const int fr = tid & 63;
  const int f = f0 + fr;
  const bool valid = f < F;
  for (int m = tid >> 6; m < n_mels; m += 4) {
    const int s = mt.first[m], cnt = mt.count[m], off = mt.offset[m];
    float acc = 0.f;
    for (int i = 0; i < cnt; ++i) acc += mt.w[off + i] * pw[fr * kPB + s + i];
    const float v = log10f(fmaxf(acc, 1e-10f));
    if (valid) {
      raw[((long)b * n_mels + m) * fcap + f] = v;
      bmax = fmaxf(bmax, v);
    }
  }
  bmax = wave_max(bmax);
  __shared__ float red[4];
  if (lane == 0) red[wave] = bmax;
  __syncthreads();
  if (tid == 0) atomicMax(&wmax[b], enc_max(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// ------------------------------------------------------------------------------------------------
// Kernel 1, FFT form (default): one workgroup = 32 consecutive frames of one window.  The 400-point real DFT of a
// frame is a two-pass Cooley-Tukey transform with N = 20 x 20 (n = 20 n1 + n2, k = k1 + 20 k2):
//   pass 1, thread per (frame, n2):  Y[n2][k1] = sum_n1 xw[20 n1 + n2] W20^(n1 k1), k1 = 0..10 (real input: the
//           other half is the conjugate), the 20 samples in registers, W20 as compile-time constants;
//   pass 2, thread per (frame, k1):  t[n2] = Y[n2][k1] W400^(n2 k1) (table in LDS), then
//           X[k1 + 20 k2] = sum_n2 t[n2] W20^(n2 k2) for the bins <= 200, and |X|^2 straight to the power image.
// ~54 kFLOP per frame on the vector ALUs instead of the 333 kFLOP of the DFT-as-GEMM (no 666 KB basis stream per
// workgroup); audio, Y (the 11 stored k1 columns, float2) and the power image all stay in LDS.
// The filterbank / log10 / per-window max tail is the GEMM form's.
// ------------------------------------------------------------------------------------------------
constexpr int kFftFrames = 32;
constexpr int kFftThreads = kFftFrames * 20;  // 10 waves: one (frame, n2) item per thread in pass 1, (frame, k1) in pass 2
constexpr int kFftSeg = kHop * (kFftFrames - 1) + kFFT;  // 5360 samples

// cos / sin(2 pi m / 20), m = 0..19 (folded into the unrolled loops as literals)
__device__ constexpr float kC20[20] = {1.0f, 0.95105651629515357f, 0.80901699437494742f, 0.58778525229247313f,
                                       0.30901699437494742f, 0.0f, -0.30901699437494742f, -0.58778525229247313f,
                                       -0.80901699437494742f, -0.95105651629515357f, -1.0f, -0.95105651629515357f,
                                       -0.80901699437494742f, -0.58778525229247313f, -0.30901699437494742f, 0.0f,
                                       0.30901699437494742f, 0.58778525229247313f, 0.80901699437494742f,
                                       0.95105651629515357f};
__device__ constexpr float kS20[20] = {0.0f, 0.30901699437494742f, 0.58778525229247313f, 0.80901699437494742f,
                                       0.95105651629515357f, 1.0f, 0.95105651629515357f, 0.80901699437494742f,
                                       0.58778525229247313f, 0.30901699437494742f, 0.0f, -0.30901699437494742f,
                                       -0.58778525229247313f, -0.80901699437494742f, -0.95105651629515357f, -1.0f,
                                       -0.95105651629515357f, -0.80901699437494742f, -0.58778525229247313f,
                                       -0.30901699437494742f};

// audio + Y (the power image reuses Y's space after pass 2) + the W400 table: 80 KB, two workgroups per CU
constexpr int kYS = 21;  // Y row stride (float2): odd, so pass 2's per-thread row reads fall in different banks
size_t logmel_fft_smem_bytes() { return (size_t)kFftSeg * 4 + (size_t)kFftFrames * 11 * kYS * 8 + 2 * kFFT * 4; }

__global__ __launch_bounds__(kFftThreads) void logmel_fft_kernel(const float* __restrict__ pcm, long stride,
                                                         const long* __restrict__ lens, MelTable mt, int n_mels,
                                                         float* __restrict__ raw, int fcap, int* __restrict__ wmax) {
  const int b = blockIdx.y;
  const long N = lens[b];
  const int F = (int)(N / kHop) + 1;
  const int f0 = blockIdx.x * kFftFrames;
  if (f0 >= F) return;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* aud = smem;                                            // [kFftSeg], Hann applied per frame in pass 1
  float2* Y = reinterpret_cast<float2*>(smem + kFftSeg);        // [frame][k1 0..10][n2 0..19, row stride kYS]
  float* pw = smem + kFftSeg;                                   // [frame][208], over Y once pass 2 has read it
  float* tc = smem + kFftSeg + kFftFrames * 11 * kYS * 2;       // cos(2 pi j / 400)
  float* ts = tc + kFFT;                                        // sin(2 pi j / 400)
  // the sparse filterbank in LDS, loaded beside the audio: the tail's per-mel reads are then LDS, not a chain of
  // dependent global loads per mel
  __shared__ int mfirst[kMaxMels], mcount[kMaxMels], moff[kMaxMels];
  __shared__ float mw[kMelWCap];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < n_mels; i += kFftThreads) {
    mfirst[i] = mt.first[i];
    mcount[i] = mt.count[i];
    moff[i] = mt.offset[i];
  }
  for (int i = tid; i < kMelWCap; i += kFftThreads) mw[i] = mt.w[i];  // (the table allocation holds n_mels x 201)
  const float* x = pcm + (long)b * stride;
  const long Lp = N + kHop;  // padded length
  const long period = 2 * (Lp - 1);
  const long j0 = (long)f0 * kHop - kFFT / 2;
  for (int i = tid; i < kFftSeg; i += kFftThreads) {
    const long j = j0 + i;
    long m = j;
    if (j < 0 || j >= Lp) {  // reflect (only the frames at the buffer edges take the 64-bit modulo)
      m = j % period;
      if (m < 0) m += period;
      if (m >= Lp) m = period - m;
    }
    aud[i] = (m < N) ? x[m] : 0.0f;
  }
  for (int j = tid; j < kFFT; j += kFftThreads) {
    float sv, cv;
    sincospif(2.0f * (float)j / (float)kFFT, &sv, &cv);
    tc[j] = cv;
    ts[j] = sv;
  }
  __syncthreads();
  // pass 1: (frame, n2) -> Y[frame][k1][n2], k1 = 0..10; periodic Hann w[n] = 0.5 - 0.5 cos(2 pi n / 400)
  for (int it = tid; it < kFftFrames * 20; it += kFftThreads) {
    const int fr = it / 20, n2 = it - fr * 20;
    float a[20];
#pragma unroll
    for (int n1 = 0; n1 < 20; ++n1) {
      const int n = 20 * n1 + n2;
      a[n1] = aud[fr * kHop + n] * (0.5f - 0.5f * tc[n]);
    }
#pragma unroll
    for (int k1 = 0; k1 <= 10; ++k1) {
      float re = 0.f, im = 0.f;
#pragma unroll
      for (int n1 = 0; n1 < 20; ++n1) {
        re = fmaf(a[n1], kC20[(n1 * k1) % 20], re);
        im = fmaf(a[n1], -kS20[(n1 * k1) % 20], im);
      }
      Y[(fr * 11 + k1) * kYS + n2] = make_float2(re, im);
    }
  }
  __syncthreads();
  // pass 2: (frame, k1) -> |X[k1 + 20 k2]|^2 for the bins <= 200 (one item per thread: kFftThreads = frames x 20)
  static_assert(kFftThreads == kFftFrames * 20, "pass 2 keeps its item's powers in registers across the barrier");
  float pv[11];
  int pfr = 0, pk1 = 0;
  {
    const int it = tid;
    const int fr = it / 20, k1 = it - fr * 20;
    pfr = fr;
    pk1 = k1;
    const bool conj = k1 > 10;
    const int kk = conj ? 20 - k1 : k1;
    float tr[20], ti[20];
#pragma unroll
    for (int n2 = 0; n2 < 20; ++n2) {
      const float2 y = Y[(fr * 11 + kk) * kYS + n2];
      const float yr = y.x, yi = conj ? -y.y : y.y;
      const int j = (n2 * k1) % kFFT;  // W400^(n2 k1) = cos - i sin
      const float c = tc[j], sn = ts[j];
      tr[n2] = yr * c + yi * sn;
      ti[n2] = yi * c - yr * sn;
    }
#pragma unroll
    for (int k2 = 0; k2 <= 10; ++k2) {
      const int k = k1 + 20 * k2;
      if (k > 200) break;
      float xr = 0.f, xi = 0.f;
#pragma unroll
      for (int n2 = 0; n2 < 20; ++n2) {
        const float c = kC20[(n2 * k2) % 20], sn = kS20[(n2 * k2) % 20];
        xr = fmaf(tr[n2], c, fmaf(ti[n2], sn, xr));
        xi = fmaf(ti[n2], c, fmaf(-tr[n2], sn, xi));
      }
      pv[k2] = xr * xr + xi * xi;
    }
  }
  __syncthreads();  // every thread has read Y: its space becomes the power image
#pragma unroll
  for (int k2 = 0; k2 <= 10; ++k2)
    if (pk1 + 20 * k2 <= 200) pw[pfr * (kBinTiles * 16) + pk1 + 20 * k2] = pv[k2];
  __syncthreads();
  // sparse filterbank + log10; thread -> (frame = tid & 31, mel stride 8)
  float bmax = -INFINITY;
  const int fr = tid & (kFftFrames - 1);
  const int f = f0 + fr;
  const bool valid = f < F;
  constexpr int kPB = kBinTiles * 16;
  for (int m = tid / kFftFrames; m < n_mels; m += kFftThreads / kFftFrames) {
    const int s0 = mfirst[m], cnt = mcount[m], off = moff[m];
    float acc = 0.f;
    for (int i = 0; i < cnt; ++i) acc += mw[off + i] * pw[fr * kPB + s0 + i];
    const float v = log10f(fmaxf(acc, 1e-10f));
    if (valid) {
      raw[((long)b * n_mels + m) * fcap + f] = v;
      bmax = fmaxf(bmax, v);
    }
  }
  bmax = wave_max(bmax);
  __shared__ float red[kFftThreads / 64];
  if (lane == 0) red[wave] = bmax;
  __syncthreads();
  if (tid == 0) {
    float mx = red[0];
    for (int w2 = 1; w2 < kFftThreads / 64; ++w2) mx = fmaxf(mx, red[w2]);
    atomicMax(&wmax[b], enc_max(mx));
  }
}

static bool logmel_use_gemm() {  // WMX_LOGMEL_GEMM=1: the DFT-as-GEMM form (A/B and parity reference runs)
  static const bool v = getenv("WMX_LOGMEL_GEMM") != nullptr;
  return v;
}

double logmel_flops_per_frame() { return logmel_use_gemm() ? 400.0 * 416 * 2 : 53600.0; }

// out[b][m][t] = (max(raw, max_b - 8) + 4) / 4 for t < segment_size, else 0
__global__ __launch_bounds__(256) void logmel_finalize_kernel(const float* __restrict__ raw, const long* __restrict__ lens,
                                                              const int* __restrict__ seek, const int* __restrict__ wmax,
                                                              int n_mels, int fcap, float* __restrict__ out, int B) {
  const long total = (long)B * n_mels * 3000;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i % 3000);
    const long bm = i / 3000;
    const int b = (int)(bm / n_mels);
    const int F = (int)(lens[b] / kHop) + 1;
    const int sk = seek ? seek[b] : 0;
    const int size = min(3000, F - 1 - sk);
    float v = 0.f;
    if (t < size) {
      const float mx = dec_max(wmax[b]);
      v = (fmaxf(raw[bm * fcap + sk + t], mx - 8.0f) + 4.0f) * 0.25f;
    }
    out[i] = v;
  }
}

size_t logmel_smem_bytes() { return (size_t)(kSeg + 2 * kKChunk * kCols) * sizeof(float); }

void launch_logmel(const float* pcm, long stride, const long* lens_dev, const int* seek_dev, int B, int max_frames,
                   const float* basis, const int* mfirst, const int* mcount, const int* moff, const float* mw,
                   int n_mels, float* raw, int fcap, int* wmax, float* out, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    WMX_HIP(hipFuncSetAttribute((const void*)logmel_raw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)logmel_smem_bytes()));
    WMX_HIP(hipFuncSetAttribute((const void*)logmel_fft_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)logmel_fft_smem_bytes()));
    attr = true;
  }
  WMX_HIP(hipMemsetD32Async((hipDeviceptr_t)wmax, (int)0x80000000, B, st));
  MelTable mt{mfirst, mcount, moff, mw};
  WMX_CHECK(n_mels <= kMaxMels, "logmel: n_mels");
  if (logmel_use_gemm()) {
    dim3 g1(cdiv(max_frames, kFramesPerWG), B);
    hipLaunchKernelGGL(logmel_raw_kernel, g1, dim3(256), logmel_smem_bytes(), st, pcm, stride, lens_dev, basis, mt,
                       n_mels, raw, fcap, wmax);
  } else {
    dim3 g1(cdiv(max_frames, kFftFrames), B);
    hipLaunchKernelGGL(logmel_fft_kernel, g1, dim3(kFftThreads), logmel_fft_smem_bytes(), st, pcm, stride, lens_dev, mt,
                       n_mels, raw, fcap, wmax);
  }
  long total = (long)B * n_mels * 3000;
  int g2 = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(logmel_finalize_kernel, dim3(g2), dim3(256), 0, st, raw, lens_dev, seek_dev, wmax, n_mels, fcap,
                     out, B);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
