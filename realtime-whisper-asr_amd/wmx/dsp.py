"""Pre-ASR DSP of the reference microphone loop, batched over streams on the GPU.

* `FilterSeparator` mirrors `SimpleFilterSeparator` (reference vocal_separation.py:303-370): an order-4 Butterworth
  band-pass (85-3400 Hz by default, config.json "vocal_separation") applied forward and backward with
  scipy.signal.filtfilt semantics; `separate(audio)` returns (vocal, background = audio - vocal).
  The filter is designed here on the host (the scipy.signal.butter / lfilter_zi algorithms restated in numpy) and
  run by `wmx_filtfilt` (fp64 recursion, one workgroup per stream).
* `AudioDeduplicator` mirrors the reference class of the same name (audio_deduplicator.py:18-330): the 5-feature
  vector of every chunk comes from `wmx_dedup_features`; the time-window history, cosine similarity and skip
  decision are host logic, as in the reference.
* `create_separator(method, sample_rate, **kw)` has the reference factory's shape (vocal_separation.py:375);
  only "filter" and "none" exist here (demucs / spleeter are out of scope: SURVEY.md §8).
"""
from __future__ import annotations

import time
from collections import deque

import numpy as np

from ._lib import check, dptr, fptr, lib, lptr


# ---------------------------------------------------------------------------------------------
# filter design: scipy.signal.butter(N, Wn, btype='band') and lfilter_zi, restated
# ---------------------------------------------------------------------------------------------
def butter_bandpass(order: int, low: float, high: float, fs: float):
    """(b, a) of scipy.signal.butter(order, [low/(fs/2), high/(fs/2)], btype='band'): analog Butterworth
    prototype -> low-pass to band-pass -> bilinear transform (fs = 2, pre-warped edges) -> polynomials."""
    wn = np.array([low, high], np.float64) / (fs / 2.0)
    p = -np.exp(1j * np.pi * np.arange(-order + 1, order, 2) / (2 * order))  # buttap
    k = 1.0
    fs2 = 2.0
    warped = 2 * fs2 * np.tan(np.pi * wn / fs2)
    bw = warped[1] - warped[0]
    wo = np.sqrt(warped[0] * warped[1])
    p_lp = p * bw / 2
    p_bp = np.concatenate([p_lp + np.sqrt(p_lp ** 2 - wo ** 2), p_lp - np.sqrt(p_lp ** 2 - wo ** 2)])
    z_bp = np.zeros(order, np.complex128)
    k_bp = k * bw ** order
    f2 = 2 * fs2  # bilinear_zpk
    z_z = (f2 + z_bp) / (f2 - z_bp)
    p_z = (f2 + p_bp) / (f2 - p_bp)
    z_z = np.append(z_z, -np.ones(len(p_bp) - len(z_bp)))
    k_z = k_bp * np.real(np.prod(f2 - z_bp) / np.prod(f2 - p_bp))
    b = np.real(k_z * np.poly(z_z))
    a = np.real(np.poly(p_z))
    return b, a


def lfilter_zi(b, a):
    """scipy.signal.lfilter_zi: steady-state initial state of the direct-form-II-transposed filter."""
    b = np.asarray(b, np.float64)
    a = np.asarray(a, np.float64)
    b, a = b / a[0], a / a[0]
    n = max(len(a), len(b))
    a = np.pad(a, (0, n - len(a)))
    b = np.pad(b, (0, n - len(b)))
    comp = np.zeros((n - 1, n - 1))
    comp[0, :] = -a[1:]
    comp[1:, :-1] += np.eye(n - 2)
    return np.linalg.solve(np.eye(n - 1) - comp.T, b[1:] - a[1:] * b[0])


def _ctx_handle(ctx):
    return ctx._h if hasattr(ctx, "_h") else ctx


def filtfilt_batch(ctx, chunks, b, a):
    """filtfilt of every 1-D chunk (any lengths > 3 * len(a)) in one launch; returns float32 arrays."""
    b = np.ascontiguousarray(b, np.float64)
    a = np.ascontiguousarray(a, np.float64)
    assert len(a) == len(b)
    zi = np.ascontiguousarray(lfilter_zi(b, a), np.float64)
    a0 = a[0]
    b, a = np.ascontiguousarray(b / a0), np.ascontiguousarray(a / a0)
    lens = np.array([len(c) for c in chunks], np.int64)
    stride = max(1, int(lens.max()))
    x = np.zeros((len(chunks), stride), np.float32)
    for i, c in enumerate(chunks):
        x[i, :len(c)] = c
    y = np.empty_like(x)
    check(lib.wmx_filtfilt(_ctx_handle(ctx), fptr(x), stride, lptr(lens), len(chunks), dptr(b), dptr(a), dptr(zi),
                           len(b), fptr(y)))
    return [y[i, :lens[i]] for i in range(len(chunks))]


def dedup_features_batch(ctx, chunks, sample_rate: int = 16000):
    """[B, 5] normalised (rms, spectral centroid, zcr, roll-off, bandwidth) of every chunk (<= 8000 samples)."""
    lens = np.array([len(c) for c in chunks], np.int64)
    stride = max(1, int(lens.max()))
    x = np.zeros((len(chunks), stride), np.float32)
    for i, c in enumerate(chunks):
        x[i, :len(c)] = c
    out = np.empty((len(chunks), 5), np.float32)
    check(lib.wmx_dedup_features(_ctx_handle(ctx), fptr(x), stride, lptr(lens), len(chunks), float(sample_rate),
                                 fptr(out)))
    return out


# ---------------------------------------------------------------------------------------------
# reference-surface mirrors
# ---------------------------------------------------------------------------------------------
class VocalSeparator:
    """vocal_separation.py:18-45: identity separator ("none")."""

    def __init__(self, sample_rate: int = 16000):
        self.sample_rate = sample_rate
        self.enabled = False

    def separate(self, audio):
        return audio, None

    def is_available(self) -> bool:
        return self.enabled


class FilterSeparator(VocalSeparator):
    """SimpleFilterSeparator (vocal_separation.py:303-370) on the GPU; `ctx` is a wmx.engine.Context."""

    def __init__(self, ctx, sample_rate: int = 16000, low_cut: float = 85.0, high_cut: float = 3400.0):
        super().__init__(sample_rate)
        self.ctx = ctx
        self.low_cut = low_cut
        self.high_cut = high_cut
        self.b, self.a = butter_bandpass(4, low_cut, high_cut, sample_rate)
        self.enabled = True

    def separate(self, audio):
        audio = np.asarray(audio, np.float32)
        if audio.ndim > 1:
            audio = np.mean(audio, axis=1).astype(np.float32)
        if len(audio) <= 3 * len(self.a):  # scipy raises here; the reference then returns the input unchanged
            return audio, None
        vocal = filtfilt_batch(self.ctx, [audio], self.b, self.a)[0]
        return vocal, audio - vocal

    def separate_batch(self, chunks):
        """One launch for the chunks of many streams; [(vocal, background)] in order."""
        chunks = [np.asarray(c, np.float32) for c in chunks]
        ok = [i for i, c in enumerate(chunks) if len(c) > 3 * len(self.a)]
        out = [(c, None) for c in chunks]
        if ok:
            ys = filtfilt_batch(self.ctx, [chunks[i] for i in ok], self.b, self.a)
            for i, y in zip(ok, ys):
                out[i] = (y, chunks[i] - y)
        return out


def create_separator(method: str = "filter", sample_rate: int = 16000, ctx=None, **kwargs):
    """vocal_separation.py:375-410 factory: "filter" -> FilterSeparator (GPU), "none"/"off" -> VocalSeparator."""
    m = method.lower()
    if m in ("none", "off"):
        return VocalSeparator(sample_rate)
    if m == "filter":
        if ctx is None:
            raise ValueError("the GPU filter separator needs a wmx Context (ctx=...)")
        return FilterSeparator(ctx, sample_rate, kwargs.get("low_cut", 85.0), kwargs.get("high_cut", 3400.0))
    raise ValueError(f"unsupported separation method {method!r} (demucs / spleeter are out of scope)")


class AudioDeduplicator:
    """audio_deduplicator.py:18-330 with the feature extraction on the GPU (`features_fn` overrides it, e.g. for
    CPU tests).  Same thresholds, time window, history bound, statistics and return values."""

    def __init__(self, ctx=None, similarity_threshold: float = 0.95, time_window: float = 3.0,
                 min_audio_length: float = 0.1, enable: bool = True, features_fn=None):
        self.ctx = ctx
        self.similarity_threshold = similarity_threshold
        self.time_window = time_window
        self.min_audio_length = min_audio_length
        self.enabled = enable
        self.feature_history = deque(maxlen=100)
        self._features_fn = features_fn
        self.reset_stats()

    def _extract_features(self, audio, sample_rate: int = 16000):
        if self._features_fn is not None:
            return self._features_fn(audio, sample_rate)
        if len(audio) == 0:
            return np.zeros(5, np.float32)
        return dedup_features_batch(self.ctx, [np.asarray(audio, np.float32)], sample_rate)[0]

    @staticmethod
    def _cosine_similarity(v1, v2) -> float:
        n1, n2 = np.linalg.norm(v1), np.linalg.norm(v2)
        if n1 < 1e-10 or n2 < 1e-10:
            return 0.0
        return float((np.dot(v1, v2) / (n1 * n2) + 1.0) / 2.0)

    def _clean_history(self, current_time: float):
        cutoff = current_time - self.time_window
        self.feature_history = deque([(f, t, n) for f, t, n in self.feature_history if t > cutoff], maxlen=100)

    def should_skip(self, audio, sample_rate: int = 16000, current_time=None, features=None):
        """audio_deduplicator.py:217-298; `features` (precomputed, e.g. by a batched launch) skips extraction."""
        if not self.enabled:
            return False, None, None
        if current_time is None:
            current_time = time.time()
        self.stats["total_checked"] += 1
        audio_length = len(audio) / sample_rate
        if audio_length < self.min_audio_length:
            self.stats["passed"] += 1
            return False, None, None
        self._clean_history(current_time)
        try:
            feats = self._extract_features(audio, sample_rate) if features is None else np.asarray(features)
        except Exception:
            self.stats["passed"] += 1
            return False, None, None
        best, best_t = 0.0, None
        for hf, ht, _ in self.feature_history:
            sim = self._cosine_similarity(feats, hf)
            if sim > best:
                best, best_t = sim, ht
        if best >= self.similarity_threshold:
            reason = "duplicate" if best >= 0.98 else "similar"
            self.stats["skipped_duplicate" if reason == "duplicate" else "skipped_similar"] += 1
            self.stats["total_audio_time_skipped"] += audio_length
            return True, reason, {"type": reason, "similarity": best,
                                  "time_since_similar": current_time - best_t if best_t else None,
                                  "audio_length": audio_length}
        self.feature_history.append((feats, current_time, audio_length))
        self.stats["passed"] += 1
        return False, None, None

    def get_stats(self):
        return dict(self.stats)

    def reset_stats(self):
        self.stats = {"total_checked": 0, "skipped_duplicate": 0, "skipped_similar": 0, "passed": 0,
                      "total_audio_time_skipped": 0.0}

    def reset(self):
        self.feature_history.clear()
        self.reset_stats()


class MicFrontEnd:
    """The per-chunk pre-ASR stage of the reference microphone loop (一键实时识别麦克风.py:1473-1500) for many
    streams at once: band-pass separation (vocal_separator.separate) then audio-level dedup (should_skip), each as
    ONE launch over all streams' chunks.  Every stream keeps its own deduplicator history.  `process` returns, per
    stream, the chunk to insert into its OnlineASRProcessor, or None when the deduplicator skipped it."""

    def __init__(self, ctx, n_streams: int, separator=None, dedup: dict | None = None, sample_rate: int = 16000):
        self.ctx = ctx
        self.sr = sample_rate
        self.separator = separator
        self.dedups = [AudioDeduplicator(ctx, **dedup) for _ in range(n_streams)] if dedup is not None else None

    def process(self, chunks, current_time=None):
        chunks = [np.asarray(c, np.float32).reshape(-1) for c in chunks]
        if self.separator is not None and self.separator.is_available():
            chunks = [v for v, _ in self.separator.separate_batch(chunks)]
        if self.dedups is None:
            return chunks
        t = time.time() if current_time is None else current_time
        idx = [i for i, c in enumerate(chunks) if 0 < len(c) <= 8000]
        feats = dedup_features_batch(self.ctx, [chunks[i] for i in idx], self.sr) if idx else []
        fmap = {i: f for i, f in zip(idx, feats)}
        out = []
        for i, c in enumerate(chunks):
            skip, _, _ = self.dedups[i].should_skip(c, self.sr, current_time=t, features=fmap.get(i))
            out.append(None if skip else c)
        return out
