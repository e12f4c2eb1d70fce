"""CPU restatement of the pre-ASR DSP of the reference microphone loop.  Test
infrastructure only (see oracle/__init__.py): the product path is wmx.dsp + csrc/wmx_dsp.hip.

* filtfilt: scipy.signal.filtfilt 1.15 defaults, as called by SimpleFilterSeparator.separate
  (reference vocal_separation.py:344-353): odd extension of padlen = 3 * max(len(a), len(b)) samples, lfilter
  (direct form II transposed, float64) forward from lfilter_zi * ext[0], backward from lfilter_zi * y[-1],
  the middle samples.  Pinned against scipy.signal itself and the reference separator's outputs
  (tests/golden/dsp_golden.npz).
* dedup_features: AudioDeduplicator._extract_features (reference audio_deduplicator.py:60-160), restated with the
  same numpy calls; pinned against the reference module's outputs (tests/golden/dsp_golden.npz).
"""
from __future__ import annotations

import numpy as np


def lfilter(b, a, x, zi):
    """Direct form II transposed, float64, one sample at a time (scipy.signal.lfilter with zi)."""
    b = np.asarray(b, np.float64) / a[0]
    a = np.asarray(a, np.float64) / a[0]
    n = len(b)
    z = np.array(zi, np.float64).copy()
    y = np.empty(len(x), np.float64)
    for i, xi in enumerate(np.asarray(x, np.float64)):
        yi = b[0] * xi + z[0]
        for k in range(n - 2):
            z[k] = b[k + 1] * xi + z[k + 1] - a[k + 1] * yi
        z[n - 2] = b[n - 1] * xi - a[n - 1] * yi
        y[i] = yi
    return y


def lfilter_zi(b, a):
    b = np.asarray(b, np.float64) / a[0]
    a = np.asarray(a, np.float64) / a[0]
    n = len(a)
    comp = np.zeros((n - 1, n - 1))
    comp[0, :] = -a[1:]
    comp[1:, :-1] += np.eye(n - 2)
    return np.linalg.solve(np.eye(n - 1) - comp.T, b[1:] - a[1:] * b[0])


def filtfilt(b, a, x):
    x = np.asarray(x, np.float64)
    padlen = 3 * max(len(a), len(b))
    if len(x) <= padlen:
        raise ValueError("input shorter than padlen")
    ext = np.concatenate([2 * x[0] - x[padlen:0:-1], x, 2 * x[-1] - x[-2:-padlen - 2:-1]])
    zi = lfilter_zi(b, a)
    y = lfilter(b, a, ext, zi * ext[0])
    y = lfilter(b, a, y[::-1], zi * y[-1])[::-1]
    return y[padlen:-padlen]


def dedup_features(audio, sample_rate: int = 16000):
    """The 5 normalised features of one chunk (audio_deduplicator.py:60-160)."""
    audio = np.asarray(audio, np.float32)
    if len(audio) == 0:
        return np.zeros(5, np.float32)
    rms = np.sqrt(np.mean(audio ** 2))
    mag = np.abs(np.fft.rfft(audio))
    freqs = np.fft.rfftfreq(len(audio), 1.0 / sample_rate)
    half = sample_rate / 2
    centroid = np.sum(freqs * mag) / (np.sum(mag) + 1e-10) / half
    zcr = np.sum(np.diff(np.signbit(audio))) / len(audio) if len(audio) > 1 else 0.0
    cs = np.cumsum(mag)
    total = cs[-1]
    if total > 1e-10:
        idx = np.where(cs >= 0.85 * total)[0]
        rolloff = freqs[idx[0]] / half if len(idx) else 1.0
    else:
        rolloff = 0.0
    if centroid > 0:
        cf = centroid * sample_rate / 2
        band = np.sqrt(np.sum(((freqs - cf) ** 2) * mag) / (np.sum(mag) + 1e-10)) / half
    else:
        band = 0.0
    f = np.array([rms, centroid, zcr, rolloff, band], np.float32)
    mx = np.max(np.abs(f))
    return f / mx if mx > 1e-10 else np.zeros(5, np.float32)
