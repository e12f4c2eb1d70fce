// Batched log-mel front end (faster-whisper 1.2.1 FeatureExtractor semantics).
//
//   x' = pcm[0..N) ++ zeros(160); frame f covers x'[160f-200, 160f+200) with numpy 'reflect' padding;
//   periodic Hann 400; |rfft|^2 (201 bins); slaney mel; log10(max(.,1e-10)); drop the last STFT frame
//   (F = N//160 + 1 frames); per-window max-8 clamp; (x+4)/4; encoder window = frames [seek, seek+3000)
//   of the first min(3000, F-1-seek) content frames, zero padded (pad_or_trim).
//
// Two launches, no memset, 13.8 MB of algorithmic HBM traffic per 4 windows moved about once (round 6):
//   logmel_fft_kernel   one workgroup = 16 consecutive frames of one window, aligned so that its frames are one
//                       16-frame block of the OUTPUT window (f0 = seek mod 16 + 16 k); writes (v + 4) / 4 of its
//                       in-window frames straight into the encoder input [B][n_mels][3000] and two statistics: the
//                       block's max of v over every frame (the per-window max runs over the whole audio) and, per mel,
//                       the min of its in-window values.  Plain stores of per-block partials: no atomics, no memset.
//   logmel_clamp_kernel one workgroup = one 16-frame output block, one thread per mel: the window max from the block
//                       maxima, then only the (mel, block) row pieces whose min lies below max - 8 are read and
//                       clamped (about 6 % of them on speech-like audio), and the pad frames are zeroed.
// Rounding: max((v + 4) / 4, (fl(gmax - 8) + 4) / 4) equals (max(v, fl(gmax - 8)) + 4) / 4 bit for bit (x -> fl(x + 4)
// is monotone, the / 4 exact), the form the previous raw + finalize pair computed.
#include "wmx_common.h"
#include "wmx_kernels.h"

namespace wmx {

constexpr int kFFT = 400, kHop = 160, kOutFrames = 3000;
constexpr int kBinsPad = 208;  // power image row stride (201 bins, padded)

// mel filter table: per mel m: first bin, count, offset into weights
struct MelTable {
  const int* first;
  const int* count;
  const int* offset;
  const float* w;
};

// ------------------------------------------------------------------------------------------------
// FFT kernel: the 400-point real DFT of a frame is a two-pass Cooley-Tukey transform with N = 20 x 20
// (n = 20 n1 + n2, k = k1 + 20 k2):
//   pass 1, thread per (frame, n2):  Y[n2][k1] = sum_n1 xw[20 n1 + n2] W20^(n1 k1), k1 = 0..10 (real input: the
//           other half is the conjugate), the 20 samples in registers, W20 as compile-time constants;
//   pass 2, thread per (frame, k1):  t[n2] = Y[n2][k1] W400^(n2 k1) (table in LDS), then
//           X[k1 + 20 k2] = sum_n2 t[n2] W20^(n2 k2) for the bins <= 200, and |X|^2 straight to the power image.
// ~54 kFLOP per frame on the vector ALUs; audio, Y (the 11 stored k1 columns, float2) and the power image stay in
// LDS.  The prologue issues every global load of the workgroup (audio as 16-byte loads on the interior path, the
// filterbank tables) before the first LDS store, so it costs one round trip.
// ------------------------------------------------------------------------------------------------
// frames per workgroup = one output block: 16 (320 threads, 47 KiB of LDS, three workgroups per CU) ran 21.2 us per 4
// windows against 30.9 for 32 (640 threads, 86 KiB, one per CU) (gpurun_out/r06p)
constexpr int kFftFrames = 16;
static_assert(kFftFrames == 16 || kFftFrames == 32, "log-mel: block size");
constexpr int kFftThreads = kFftFrames * 20;  // one (frame, n2) item per thread in pass 1, (frame, k1) in pass 2
constexpr int kFftSeg = kHop * (kFftFrames - 1) + kFFT;  // 5360 / 2800 samples
constexpr int kSegVec = kFftSeg / 4;                      // 16-byte pieces
static_assert(2 * kFftThreads < kSegVec && kSegVec <= 3 * kFftThreads, "interior audio: three 16-byte loads per thread");

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

// audio + Y (the power image reuses Y's space after pass 2) + the W400 table: 42.9 KiB at 16 frames, three per CU
constexpr int kYS = 21;  // Y row stride (float2): odd, so pass 2's per-thread row reads fall in different banks
constexpr size_t kFftLdsUsed = (size_t)kFftSeg * 4 + (size_t)kFftFrames * 11 * kYS * 8 + 2 * kFFT * 4;  // 42.9 KiB at 16
// Co-residency (round 6, tools/conc_probe4.py / conc_probe6.py): built with the compiler's SLP vectorizer, which packs
// this kernel's f32 arithmetic into v_pk_fma/add/mul_f32, a workgroup sharing its CU with another context's MFMA GEMM
// (gemm_kernel, with or without LDS-DMA staging) returned wrong spectra for a few frames in 4-17 of 15 calls -- the
// frames whose (frame, n2) item group starts in the upper half of a wave -- although both kernels address only their
// own LDS; alone on the CU, 0 of 15.  Built without it (the Makefile compiles this file with -fno-slp-vectorize: no
// packed f32 VALU), 0 of 60 calls differ while sharing CUs, 16- and 32-frame blocks alike (gpurun_out/r06o, r06p).
size_t logmel_fft_smem_bytes() { return kFftLdsUsed; }

// min over each aligned group of kFftFrames lanes (16: one DPP row; 32: two rows joined by permlane16_swap)
__device__ inline float block_min(float v) {
  v = fminf(v, dpp_mov<kDppXor1>(v));
  v = fminf(v, dpp_mov<kDppXor2>(v));
  v = fminf(v, dpp_mov<kDppHalfMirror>(v));
  v = fminf(v, dpp_mov<kDppMirror>(v));
  if constexpr (kFftFrames == 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  return v;
}

// the window's geometry: F STFT frames (the last one dropped from the output), content size of the output window,
// its first frame; output block k of window b is frames f0(k) = fbase + kFftFrames k, fbase = (seek mod kFftFrames) -
// kFftFrames (0 when seek is a multiple), so that the blocks align with the output window's frames
struct MelWin {
  int F, sk, size, fbase;
};
__device__ inline MelWin mel_win(const long* lens, const int* seek, int b) {
  MelWin w;
  w.F = (int)(lens[b] / kHop) + 1;
  w.sk = seek ? seek[b] : 0;
  w.size = max(0, min(kOutFrames, w.F - 1 - w.sk));
  const int fb = w.sk & (kFftFrames - 1);
  w.fbase = fb ? fb - kFftFrames : 0;
  return w;
}

// stats: [B][nblk] block maxima of v, then [B][nblk][n_mels] per-mel minima of the in-window (v + 4) / 4
__global__ __launch_bounds__(kFftThreads) void logmel_fft_kernel(const float* __restrict__ pcm, long stride,
                                                                 const long* __restrict__ lens,
                                                                 const int* __restrict__ seek, MelTable mt, int n_mels,
                                                                 float* __restrict__ out, float* __restrict__ stats,
                                                                 int nblk) {
  const int b = blockIdx.y, blk = blockIdx.x, B = gridDim.y;
  const MelWin win = mel_win(lens, seek, b);
  const long N = lens[b];
  const int F = win.F;
  const int f0 = win.fbase + kFftFrames * blk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* smax = stats + (long)b * nblk + blk;
  float* smin = stats + (long)B * nblk + ((long)b * nblk + blk) * n_mels;
  if (f0 >= F) {  // past the audio: neutral statistics (the clamp kernel reads every block of the window)
    if (tid == 0) *smax = -INFINITY;
    for (int m = tid; m < n_mels; m += kFftThreads) smin[m] = INFINITY;
    return;
  }
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* aud = smem;                                            // [kFftSeg], Hann applied per frame in pass 1
  float2* Y = reinterpret_cast<float2*>(smem + kFftSeg);        // [frame][k1 0..10][n2 0..19, row stride kYS]
  float* pw = smem + kFftSeg;                                   // [frame][208], over Y once pass 2 has read it
  float* tc = smem + kFftSeg + kFftFrames * 11 * kYS * 2;       // cos(2 pi j / 400)
  float* ts = tc + kFFT;                                        // sin(2 pi j / 400)
  // the sparse filterbank in LDS: the tail's per-mel reads are then LDS, not a chain of dependent global loads
  __shared__ int mfirst[kMaxMels], mcount[kMaxMels], moff[kMaxMels];
  __shared__ float mw[kMelWCap];
  // ---- prologue: every global load first (one round trip), then the LDS stores ----
  const float* x = pcm + (long)b * stride;
  const long j0 = (long)f0 * kHop - kFFT / 2;  // a multiple of 4 (f0 160 - 200)
  const bool interior = j0 >= 0 && j0 + kFftSeg <= N && (((uintptr_t)(x + j0)) & 15) == 0;
  // the filterbank tables first (both paths), then the audio: every global load of the workgroup in flight together
  int tf = 0, tcn = 0, to = 0;
  if (tid < n_mels) {
    tf = mt.first[tid];
    tcn = mt.count[tid];
    to = mt.offset[tid];
  }
  static_assert(kMaxMels <= kFftThreads && kMelWCap <= 2 * kFftThreads, "log-mel: table loads per thread");
  // (the table allocation holds n_mels x 201 >= kMelWCap floats)
  const float tw = mt.w[min(tid, kMelWCap - 1)];
  const float tw2 = mt.w[min(tid + kFftThreads, kMelWCap - 1)];
  if (interior) {
    const float4* xv = reinterpret_cast<const float4*>(x + j0);
    const float4 a0 = xv[tid], a1 = xv[tid + kFftThreads], a2 = xv[min(tid + 2 * kFftThreads, kSegVec - 1)];
    float4* av = reinterpret_cast<float4*>(aud);
    av[tid] = a0;
    av[tid + kFftThreads] = a1;
    if (tid + 2 * kFftThreads < kSegVec) av[tid + 2 * kFftThreads] = a2;
  } else {  // the window's edge blocks (and unaligned rows): reflect / zero padding, sample by sample
    const long Lp = N + kHop;  // padded length
    const long period = 2 * (Lp - 1);
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
  }
  for (int j = tid; j < kFFT; j += kFftThreads) {  // the W400 table
    float sv, cv;
    sincospif(2.0f * (float)j / (float)kFFT, &sv, &cv);
    tc[j] = cv;
    ts[j] = sv;
  }
  if (tid < n_mels) {
    mfirst[tid] = tf;
    mcount[tid] = tcn;
    moff[tid] = to;
  }
  if (tid < kMelWCap) mw[tid] = tw;
  if (tid + kFftThreads < kMelWCap) mw[tid + kFftThreads] = tw2;
  __syncthreads();
  // pass 1: (frame, n2) -> Y[frame][k1][n2], k1 = 0..10; periodic Hann w[n] = 0.5 - 0.5 cos(2 pi n / 400)
  {
    const int fr = tid / 20, n2 = tid - fr * 20;
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
  const int pfr = tid / 20, pk1 = tid - pfr * 20;
  {
    const bool conj = pk1 > 10;
    const int kk = conj ? 20 - pk1 : pk1;
    float tr[20], ti[20];
#pragma unroll
    for (int n2 = 0; n2 < 20; ++n2) {
      const float2 y = Y[(pfr * 11 + kk) * kYS + n2];
      const float yr = y.x, yi = conj ? -y.y : y.y;
      const int j = (n2 * pk1) % kFFT;  // W400^(n2 k1) = cos - i sin
      const float c = tc[j], sn = ts[j];
      tr[n2] = yr * c + yi * sn;
      ti[n2] = yi * c - yr * sn;
    }
#pragma unroll
    for (int k2 = 0; k2 <= 10; ++k2) {
      // (k2 = 10 holds bin 200 for k1 = 0 only; the others compute a discarded value: no branch, so pv stays in
      // registers)
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
    if (pk1 + 20 * k2 <= 200) pw[pfr * kBinsPad + pk1 + 20 * k2] = pv[k2];
  __syncthreads();
  // sparse filterbank + log10; thread -> (frame = tid mod kFftFrames, mel = tid / kFftFrames + 20 it); a mel's frames
  // are one aligned lane group, so its in-window min is a lane reduction (every lane of the wave takes part)
  float bmax = -INFINITY;
  const int fr = tid & (kFftFrames - 1);
  const int f = f0 + fr;
  const int t = f - win.sk;
  const bool valid = f >= 0 && f < F;
  const bool inwin = valid && t >= 0 && t < win.size;
  const int iters = (n_mels + kFftThreads / kFftFrames - 1) / (kFftThreads / kFftFrames);
  for (int it = 0; it < iters; ++it) {
    const int m = tid / kFftFrames + it * (kFftThreads / kFftFrames);
    float vn = INFINITY;
    if (m < n_mels) {
      const int s0 = mfirst[m], cnt = mcount[m], off = moff[m];
      float acc = 0.f;
      for (int i = 0; i < cnt; ++i) acc += mw[off + i] * pw[fr * kBinsPad + s0 + i];
      const float v = log10f(fmaxf(acc, 1e-10f));
      if (valid) bmax = fmaxf(bmax, v);
      if (inwin) {
        vn = (v + 4.0f) * 0.25f;
        out[((long)b * n_mels + m) * kOutFrames + t] = vn;
      }
    }
    const float mn = block_min(vn);
    if (m < n_mels && fr == 0) smin[m] = mn;
  }
  bmax = wave_max(bmax);
  __shared__ float red[kFftThreads / 64];
  if (lane == 0) red[wave] = bmax;
  __syncthreads();
  if (tid == 0) {
    float mx = red[0];
    for (int w2 = 1; w2 < kFftThreads / 64; ++w2) mx = fmaxf(mx, red[w2]);
    *smax = mx;
  }
}

double logmel_flops_per_frame() { return 53600.0; }

// one workgroup per (kFftFrames-frame output block, window), one thread per mel
__global__ __launch_bounds__(128) void logmel_clamp_kernel(const long* __restrict__ lens, const int* __restrict__ seek,
                                                           int n_mels, const float* __restrict__ stats, int nblk,
                                                           float* __restrict__ out) {
  const int b = blockIdx.y, j = blockIdx.x, B = gridDim.y;
  const MelWin win = mel_win(lens, seek, b);
  const int tid = threadIdx.x;
  // the window max over every block of the window
  float mx = -INFINITY;
  for (int i = tid; i < nblk; i += 128) mx = fmaxf(mx, stats[(long)b * nblk + i]);
  mx = wave_max(mx);
  __shared__ float red[2];
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  const float gmax = fmaxf(red[0], red[1]);
  const float thr = (gmax - 8.0f + 4.0f) * 0.25f;  // (fl(gmax - 8) + 4) / 4
  const int t0 = kFftFrames * j, t1 = min(t0 + kFftFrames, kOutFrames);
  // output block j is the fft kernel's block k = j + the blocks before the window's first frame
  const int k = j + (win.sk - win.fbase) / kFftFrames;
  for (int m = tid; m < n_mels; m += 128) {
    float* row = out + ((long)b * n_mels + m) * kOutFrames;
    for (int t = max(t0, win.size); t < t1; ++t) row[t] = 0.f;  // pad_or_trim
    if (t0 < win.size && k < nblk && stats[(long)B * nblk + ((long)b * nblk + k) * n_mels + m] < thr) {
      for (int t = t0; t < min(t1, win.size); ++t) row[t] = fmaxf(row[t], thr);
    }
  }
}

int logmel_blocks(int max_frames) { return (max_frames + kFftFrames - 1) / kFftFrames + 1; }

void launch_logmel(const float* pcm, long stride, const long* lens_dev, const int* seek_dev, int B, int max_frames,
                   const int* mfirst, const int* mcount, const int* moff, const float* mw, int n_mels, float* stats,
                   long stats_cap, float* out, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    WMX_HIP(hipFuncSetAttribute((const void*)logmel_fft_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)logmel_fft_smem_bytes()));
    attr = true;
  }
  WMX_CHECK(n_mels <= kMaxMels, "logmel: n_mels");
  const int nblk = logmel_blocks(max_frames);
  WMX_CHECK((long)B * nblk * (1 + n_mels) <= stats_cap, "logmel: statistics buffer too small");
  hipLaunchKernelGGL(logmel_fft_kernel, dim3(nblk, B), dim3(kFftThreads), logmel_fft_smem_bytes(), st, pcm, stride,
                     lens_dev, seek_dev, MelTable{mfirst, mcount, moff, mw}, n_mels, out, stats, nblk);
  hipLaunchKernelGGL(logmel_clamp_kernel, dim3(cdiv(kOutFrames, kFftFrames), B), dim3(128), 0, st, lens_dev, seek_dev, n_mels,
                     stats, nblk, out);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
