// Batched log-mel front end (faster-whisper 1.2.1 FeatureExtractor semantics).
//
//   x' = pcm[0..N) ++ zeros(160); frame f covers x'[160f-200, 160f+200) with numpy 'reflect' padding;
//   periodic Hann 400; |rfft|^2 (201 bins); slaney mel; log10(max(.,1e-10)); drop the last STFT frame
//   (F = N//160 + 1 frames); per-window max-8 clamp; (x+4)/4; encoder window = frames [seek, seek+3000)
//   of the first min(3000, F-1-seek) content frames, zero padded (pad_or_trim).
//
// Kernel 1 (logmel_raw): one workgroup = 64 consecutive frames of one window, 4 waves x 16 frames.
//   The windowed real DFT is a [frames x 400] x [400 x 416] f32 GEMM on v_mfma_f32_16x16x4_f32 (exact
//   fp32 FMA chains; bf16 would miss the 1e-4 gate).  Audio for the 64 frames (10480 samples, reflect
//   applied) is staged once in LDS; the Hann-folded cos/sin basis streams through LDS in 16-sample
//   K-chunks.  Re/Im tiles of one bin block share a lane layout, so |X|^2 is formed in registers,
//   written to LDS, reduced through the sparse slaney filterbank, log10'd, stored, and the block max
//   is folded into a per-window atomicMax.
// Kernel 2 (logmel_finalize): clamp, scale, slice [seek, seek+3000) and zero-pad.  HBM-bound.
#include "wmx_common.h"

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
    attr = true;
  }
  WMX_HIP(hipMemsetD32Async((hipDeviceptr_t)wmax, (int)0x80000000, B, st));
  MelTable mt{mfirst, mcount, moff, mw};
  dim3 g1(cdiv(max_frames, kFramesPerWG), B);
  hipLaunchKernelGGL(logmel_raw_kernel, g1, dim3(256), logmel_smem_bytes(), st, pcm, stride, lens_dev, basis, mt,
                     n_mels, raw, fcap, wmax);
  long total = (long)B * n_mels * 3000;
  int g2 = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(logmel_finalize_kernel, dim3(g2), dim3(256), 0, st, raw, lens_dev, seek_dev, wmax, n_mels, fcap,
                     out, B);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
