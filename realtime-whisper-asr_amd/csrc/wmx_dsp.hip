// Pre-ASR DSP of the reference's microphone loop, batched over streams:
//
//  * band-pass "vocal separation" (reference vocal_separation.py:335-358, SimpleFilterSeparator.separate):
//    scipy.signal.filtfilt(b, a, x) of an order-4 Butterworth band-pass (8th-order b, a), i.e. odd extension by
//    padlen = 3 * max(len(a), len(b)) samples at both ends, a forward lfilter started from lfilter_zi(b, a) * ext[0]
//    (direct form II transposed), a backward lfilter started from lfilter_zi * y[-1], and the middle n samples.
//    One workgroup per stream: the padded sequence streams through LDS in chunks (coalesced loads / stores by all
//    lanes) while one lane runs the recursion in fp64, as scipy does.
//  * audio-dedup features (reference audio_deduplicator.py:60-160, AudioDeduplicator._extract_features):
//    rms, spectral centroid, zero-crossing rate, 85 % spectral roll-off and spectral bandwidth of |rfft(x)|,
//    normalised by their max |.|.  One workgroup per stream: samples staged in LDS, one thread per rfft bin
//    (phasor recurrence in fp64, re-seeded every 512 samples), block reductions, the roll-off scan in bin order.
#include "wmx_common.h"
#include "wmx_kernels.h"

namespace wmx {

constexpr int kDspChunk = 2048;  // doubles of the padded sequence resident in LDS per step

__global__ __launch_bounds__(64) void filtfilt_kernel(const float* __restrict__ x, long xstride,
                                                      const long* __restrict__ lens, IIRCoefs f,
                                                      double* __restrict__ scratch, long sstride,
                                                      float* __restrict__ y, long ystride) {
  const int s = blockIdx.x, tid = threadIdx.x;
  const long n = lens[s];
  const int P = f.padlen;
  const long L = n + 2L * P;
  const float* xs = x + (long)s * xstride;
  double* e = scratch + (long)s * sstride;
  __shared__ double buf[kDspChunk];
  if (n <= P) {  // scipy raises for len(x) <= padlen; the host checks, pass the input through
    for (long i = tid; i < n; i += 64) y[(long)s * ystride + i] = xs[i];
    return;
  }
  // odd extension: [2 x0 - x[P..1], x, 2 x[n-1] - x[n-2 .. n-1-P]]
  const double x0 = xs[0], xn = xs[n - 1];
  for (long i = tid; i < L; i += 64) {
    double v;
    if (i < P)
      v = 2.0 * x0 - (double)xs[P - i];
    else if (i < P + n)
      v = (double)xs[i - P];
    else
      v = 2.0 * xn - (double)xs[n - 2 - (i - P - n)];
    e[i] = v;
  }
  const int nz = f.ntaps - 1;
  double z[kMaxTaps - 1];
  for (int pass = 0; pass < 2; ++pass) {
    __syncthreads();
    // initial state zi * (first sample of this pass' direction)
    const double first = pass == 0 ? e[0] : e[L - 1];
#pragma unroll
    for (int k = 0; k < kMaxTaps - 1; ++k) z[k] = k < nz ? f.zi[k] * first : 0.0;
    for (long c0 = 0; c0 < L; c0 += kDspChunk) {
      const int cn = (int)min((long)kDspChunk, L - c0);
      // chunk c0 of the pass' direction; backward pass walks the sequence from the end
      const long base = pass == 0 ? c0 : L - c0 - cn;
      __syncthreads();
      for (int i = tid; i < cn; i += 64) buf[i] = e[base + i];
      __syncthreads();
      if (tid == 0) {
        for (int j = 0; j < cn; ++j) {
          const int i = pass == 0 ? j : cn - 1 - j;
          const double xi = buf[i];
          const double yi = f.b[0] * xi + z[0];
#pragma unroll
          for (int k = 0; k < kMaxTaps - 2; ++k)
            if (k + 1 < nz) z[k] = f.b[k + 1] * xi + z[k + 1] - f.a[k + 1] * yi;
          // last state element
#pragma unroll
          for (int k = 0; k < kMaxTaps - 1; ++k)
            if (k == nz - 1) z[k] = f.b[k + 1] * xi - f.a[k + 1] * yi;
          buf[i] = yi;
        }
      }
      __syncthreads();
      for (int i = tid; i < cn; i += 64) e[base + i] = buf[i];
    }
  }
  __syncthreads();
  for (long i = tid; i < n; i += 64) y[(long)s * ystride + i] = (float)e[P + i];
}

void launch_filtfilt(const float* x, long xstride, const long* lens_dev, int B, const IIRCoefs& f, double* scratch,
                     long sstride, float* y, long ystride, hipStream_t st) {
  WMX_CHECK(f.ntaps >= 2 && f.ntaps <= kMaxTaps, "filtfilt: filter order");
  hipLaunchKernelGGL(filtfilt_kernel, dim3(B), dim3(64), 0, st, x, xstride, lens_dev, f, scratch, sstride, y, ystride);
  WMX_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
constexpr int kDedupThreads = 256;

__device__ inline double block_sum_d(double v, double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kDedupThreads / 64; ++w) t += red[w];
  return t;
}

__global__ __launch_bounds__(kDedupThreads) void dedup_features_kernel(const float* __restrict__ x, long xstride,
                                                                       const long* __restrict__ lens, float sr,
                                                                       float* __restrict__ feats) {
  const int s = blockIdx.x, tid = threadIdx.x;
  const int n = (int)lens[s];
  const float* xs = x + (long)s * xstride;
  __shared__ float xsh[kDedupMaxN];
  __shared__ double mag[kDedupMaxN / 2 + 1];
  __shared__ double red[kDedupThreads / 64];
  __shared__ int rolloff_idx;
  float* out = feats + (long)s * 5;
  if (n <= 0) {
    if (tid < 5) out[tid] = 0.f;
    return;
  }
  double sq = 0.0, zc = 0.0;
  for (int i = tid; i < n; i += kDedupThreads) {
    const float v = xs[i];
    xsh[i] = v;
    sq += (double)v * v;
  }
  __syncthreads();
  for (int i = tid; i + 1 < n; i += kDedupThreads) zc += (signbit(xsh[i]) != signbit(xsh[i + 1])) ? 1.0 : 0.0;
  const double sumsq = block_sum_d(sq, red);
  const double nzc = block_sum_d(zc, red);
  // |rfft| per bin: phasor recurrence exp(-2 pi i k t / n), re-seeded exactly every 512 samples
  const int nb = n / 2 + 1;
  for (int k = tid; k < nb; k += kDedupThreads) {
    double re = 0.0, im = 0.0;
    for (int t0 = 0; t0 < n; t0 += 512) {
      double sp, cp, sw, cw;
      sincospi(-2.0 * (double)(((long)k * t0) % n) / n, &sp, &cp);
      sincospi(-2.0 * (double)k / n, &sw, &cw);
      const int t1 = min(n, t0 + 512);
      for (int t = t0; t < t1; ++t) {
        const double v = xsh[t];
        re += v * cp;
        im += v * sp;
        const double c2 = cp * cw - sp * sw;
        sp = sp * cw + cp * sw;
        cp = c2;
      }
    }
    mag[k] = sqrt(re * re + im * im);
  }
  __syncthreads();
  const double df = (double)sr / n;  // rfftfreq spacing
  double m = 0.0, fm = 0.0;
  for (int k = tid; k < nb; k += kDedupThreads) {
    m += mag[k];
    fm += (k * df) * mag[k];
  }
  const double msum = block_sum_d(m, red);
  const double fmsum = block_sum_d(fm, red);
  const double half = sr / 2.0;
  const double centroid = fmsum / (msum + 1e-10) / half;
  // roll-off: first bin whose running sum (bin order, as numpy cumsum) reaches 85 % of the total
  if (tid == 0) {
    double cs = 0.0;
    int idx = -1;
    double total = 0.0;
    for (int k = 0; k < nb; ++k) total += mag[k];
    for (int k = 0; k < nb; ++k) {
      cs += mag[k];
      if (cs >= 0.85 * total) {
        idx = k;
        break;
      }
    }
    rolloff_idx = total > 1e-10 ? idx : -2;
  }
  double bw = 0.0;
  const double cf = centroid * half;
  for (int k = tid; k < nb; k += kDedupThreads) {
    const double d = k * df - cf;
    bw += d * d * mag[k];
  }
  const double bwsum = block_sum_d(bw, red);
  if (tid == 0) {
    const double rms = sqrt(sumsq / n);
    const double zcr = n > 1 ? nzc / n : 0.0;
    const double roll = rolloff_idx >= 0 ? (rolloff_idx * df) / half : (rolloff_idx == -1 ? 1.0 : 0.0);
    const double band = centroid > 0 ? sqrt(bwsum / (msum + 1e-10)) / half : 0.0;
    float v[5] = {(float)rms, (float)centroid, (float)zcr, (float)roll, (float)band};
    float mx = 0.f;
    for (int i = 0; i < 5; ++i) mx = fmaxf(mx, fabsf(v[i]));
    for (int i = 0; i < 5; ++i) out[i] = mx > 1e-10f ? v[i] / mx : 0.f;
  }
}

void launch_dedup_features(const float* x, long xstride, const long* lens_dev, int B, float sr, float* feats,
                           hipStream_t st) {
  hipLaunchKernelGGL(dedup_features_kernel, dim3(B), dim3(kDedupThreads), 0, st, x, xstride, lens_dev, sr, feats);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
