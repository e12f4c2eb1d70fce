"""Silero VAD v5 (16 kHz) on the GPU, batched over streams.

The reference fetches the network with torch.hub (asr_components.py:96) and calls it once per 512-sample window
from whisper_streaming's VADIterator (`self.model(x, self.sampling_rate).item()`, then `self.model.reset_states()`
on reset; DynamicVADIterator wraps it at asr_components.py:12-78).  Here:

* `SileroVADEngine` owns the device weights (f32) and the per-slot state (LSTM h / c, the 64-sample context) of up
  to `max_streams` streams; `process({slot: pcm})` runs every stream's pending windows in two launches
  (`wmx_vad_process`: all windows' STFT + encoder in parallel, then one workgroup per stream steps the LSTM
  through its windows in order).
* `SileroVAD` is the model object VADIterator expects: `vad(x, 16000) -> float` on exactly 512 samples (the v5
  model raises on other sizes too) and `reset_states()`.  Several `SileroVAD`s can share one engine (one slot
  each); `StreamVAD.step` batches many streams' windows into one call.

Weights: the v5 state-dict names (`tensor_shapes()`), loaded from a safetensors file when the user has one
(`load_state_dict`), else `synthetic_state_dict(seed)` (a Hann-windowed DFT basis, PyTorch-style uniform
init for the rest).  No Silero checkpoint exists in this image, so every measurement uses the synthetic weights.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, fptr, iptr, lib

WINDOW, CONTEXT, NFFT, HIDDEN, SAMPLE_RATE = 512, 64, 256, 128, 16000
ENCODER = ((129, 128, 1), (128, 64, 2), (64, 64, 2), (64, 128, 1))


def tensor_shapes():
    s = {"stft.forward_basis_buffer": (2 * (NFFT // 2 + 1), 1, NFFT)}
    for i, (ci, co, _) in enumerate(ENCODER):
        s[f"encoder.{i}.reparam_conv.weight"] = (co, ci, 3)
        s[f"encoder.{i}.reparam_conv.bias"] = (co,)
    s["decoder.rnn.weight_ih"] = (4 * HIDDEN, HIDDEN)
    s["decoder.rnn.weight_hh"] = (4 * HIDDEN, HIDDEN)
    s["decoder.rnn.bias_ih"] = (4 * HIDDEN,)
    s["decoder.rnn.bias_hh"] = (4 * HIDDEN,)
    s["decoder.decoder.2.weight"] = (1, HIDDEN, 1)
    s["decoder.decoder.2.bias"] = (1,)
    return s


def stft_basis():
    """[258, 1, 256]: rows k < 129 = Re, rows 129 + k = Im of the DFT row k (np.fft.fft(np.eye(256))), times a
    periodic Hann window -- the STFT-as-conv basis an STFT module of this shape builds."""
    n = np.arange(NFFT)
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / NFFT)
    k = np.arange(NFFT // 2 + 1)[:, None]
    ang = 2 * np.pi * k * n[None, :] / NFFT
    basis = np.concatenate([np.cos(ang), -np.sin(ang)], axis=0) * win[None, :]
    return basis[:, None, :].astype(np.float32)


def synthetic_state_dict(seed: int = 0):
    """PyTorch default init bounds: uniform(+-1/sqrt(fan_in)) with fan_in = Cin * 3 for the encoder convs, the hidden
    size for the LSTM cell and the 1x1 output conv."""
    rng = np.random.default_rng(seed)
    shapes = tensor_shapes()
    out = {"stft.forward_basis_buffer": stft_basis()}
    for name, shp in shapes.items():
        if name in out:
            continue
        layer = name.rsplit(".", 1)[0]
        fan_in = shapes[layer + ".weight"][1] * 3 if layer.startswith("encoder.") else HIDDEN
        bound = 1.0 / np.sqrt(fan_in)
        out[name] = rng.uniform(-bound, bound, size=shp).astype(np.float32)
    return out


def load_state_dict(path: str):
    """Silero v5 weights from a safetensors file (keys with or without the `_model.` prefix; 16 kHz branch)."""
    from safetensors.numpy import load_file
    raw = load_file(path)
    want = tensor_shapes()
    out = {}
    for k, v in raw.items():
        k2 = k[len("_model."):] if k.startswith("_model.") else k
        if k2 in want:
            out[k2] = np.asarray(v, np.float32).reshape(want[k2])
    missing = sorted(set(want) - set(out))
    if missing:
        raise KeyError(f"Silero state dict is missing {missing}")
    return out


class SileroVADEngine:
    """Device weights + per-slot VAD state for up to `max_streams` streams, `max_windows` windows per call."""

    def __init__(self, state_dict=None, device: int = 0, max_streams: int = 64, max_windows: int = 64):
        self.max_streams, self.max_windows = max_streams, max_windows
        h = C.c_void_p()
        check(lib.wmx_vad_create(device, max_streams, max_windows, C.byref(h)))
        self._h = h
        sd = synthetic_state_dict(0) if state_dict is None else state_dict
        for name, shp in tensor_shapes().items():
            a = np.ascontiguousarray(np.asarray(sd[name], np.float32).reshape(-1))
            assert a.size == int(np.prod(shp)), name
            check(lib.wmx_vad_set_tensor(self._h, name.encode(), fptr(a), a.size))

    def close(self):
        if getattr(self, "_h", None):
            lib.wmx_vad_free(self._h)
            self._h = None

    __del__ = close

    def reset(self, slot: int = -1):
        check(lib.wmx_vad_reset(self._h, int(slot)))

    def process(self, chunks):
        """{slot: pcm (k * 512 samples, same k for every slot)} -> {slot: probs [k]}; windows of a slot in order."""
        slots = np.array(sorted(chunks), np.int32)
        if len(slots) == 0:
            return {}
        lens = {len(chunks[s]) for s in slots}
        if len(lens) != 1:
            raise ValueError("every stream of one call carries the same number of samples")
        n = lens.pop()
        if n == 0 or n % WINDOW:
            raise ValueError(f"Provided number of samples is {n} (Supported values: multiples of {WINDOW} for 16000 "
                             "sample rate)")
        W = n // WINDOW
        x = np.ascontiguousarray(np.stack([np.asarray(chunks[s], np.float32) for s in slots]))
        probs = np.empty((len(slots), W), np.float32)
        check(lib.wmx_vad_process(self._h, fptr(x), n, iptr(slots), len(slots), W, fptr(probs)))
        return {int(s): probs[i] for i, s in enumerate(slots)}


class SileroVAD:
    """The `model` object of VADIterator (asr_components.py:23, whisper_streaming silero_vad_iterator.py): one slot of
    a shared engine; `__call__(x, sr)` -> speech probability of exactly 512 samples at 16 kHz."""

    def __init__(self, engine: SileroVADEngine | None = None, slot: int = 0):
        self.engine = engine or SileroVADEngine(max_streams=1, max_windows=8)
        self.slot = slot
        self.engine.reset(slot)

    def reset_states(self, batch_size: int = 1):
        self.engine.reset(self.slot)

    def __call__(self, x, sr: int = SAMPLE_RATE):
        if sr != SAMPLE_RATE:
            raise ValueError("Supported sampling rates: [16000] (8 kHz branch not built)")
        x = np.asarray(x.detach().cpu().numpy() if hasattr(x, "detach") else x, np.float32).reshape(-1)
        if len(x) != WINDOW:
            raise ValueError(f"Provided number of samples is {len(x)} (Supported values: 512 for 16000 sample rate)")
        return float(self.engine.process({self.slot: x})[self.slot][0])


class StreamVAD:
    """Many streams' VAD in one call per tick: `step({slot: new audio})` buffers each stream's samples, runs every
    whole 512-sample window pending on all streams (grouped by window count, one engine call per group), and
    returns {slot: probs of the windows just run}."""

    def __init__(self, engine: SileroVADEngine):
        self.engine = engine
        self.pending = {}

    def reset(self, slot: int):
        self.pending.pop(slot, None)
        self.engine.reset(slot)

    def step(self, audio):
        for s, a in audio.items():
            self.pending[s] = np.concatenate([self.pending.get(s, np.zeros(0, np.float32)),
                                              np.asarray(a, np.float32)])
        groups = {}
        for s, buf in self.pending.items():
            k = min(len(buf) // WINDOW, self.engine.max_windows)
            if k:
                groups.setdefault(k, []).append(s)
        out = {}
        for k, slots in groups.items():
            res = self.engine.process({s: self.pending[s][:k * WINDOW] for s in slots})
            for s in slots:
                self.pending[s] = self.pending[s][k * WINDOW:]
                out[s] = res[s]
        return out


def silero_model(spec: str = "silero", engine: SileroVADEngine | None = None, slot: int = 0) -> SileroVAD:
    """The VAD model a VAC processor asks for by name: "silero" = synthetic weights, else a .safetensors path."""
    if engine is None:
        sd = None if spec == "silero" else load_state_dict(spec)
        engine = SileroVADEngine(sd, max_streams=max(1, slot + 1), max_windows=8)
    return SileroVAD(engine, slot)


# ---------------------------------------------------------------------------------------------
# faster-whisper's `vad_filter=True` (the reference's CustomFasterWhisperASR.use_vad, asr_components.py:307-309):
# vad.py get_speech_timestamps / collect_chunks / SpeechTimestampsMap of faster-whisper 1.2.1, restated (the
# package is not installed here, so this is parity unpinned), with the speech probabilities from the device network
# ---------------------------------------------------------------------------------------------
VAD_DEFAULTS = dict(threshold=0.5, neg_threshold=None, min_speech_duration_ms=0, max_speech_duration_s=float("inf"),
                    min_silence_duration_ms=2000, speech_pad_ms=400)


def speech_probs(engine: SileroVADEngine, audio, slot: int = 0):
    """Per-512-sample-window probabilities of a whole buffer (zero-padded to whole windows), from a reset state:
    faster-whisper's SileroVADModel.__call__ (each window prefixed by the previous window's last 64 samples)."""
    audio = np.asarray(audio, np.float32)
    n = len(audio)
    padded = np.pad(audio, (0, WINDOW - n % WINDOW))
    engine.reset(slot)
    out = []
    per = engine.max_windows * WINDOW
    for i in range(0, len(padded), per):
        out.append(engine.process({slot: padded[i:i + per]})[slot])
    return np.concatenate(out) if out else np.zeros(0, np.float32)


def get_speech_timestamps(probs, n_samples: int, sampling_rate: int = SAMPLE_RATE, **opts):
    """faster-whisper vad.get_speech_timestamps on given window probabilities -> [{"start", "end"}] in samples."""
    o = dict(VAD_DEFAULTS)
    unknown = set(opts) - set(o)
    if unknown:
        raise TypeError(f"unknown VAD options {sorted(unknown)}")
    o.update(opts)
    threshold = o["threshold"]
    neg_threshold = o["neg_threshold"] if o["neg_threshold"] is not None else max(threshold - 0.15, 0.01)
    ws = WINDOW
    min_speech_samples = sampling_rate * o["min_speech_duration_ms"] / 1000
    speech_pad_samples = sampling_rate * o["speech_pad_ms"] / 1000
    max_speech_samples = sampling_rate * o["max_speech_duration_s"] - ws - 2 * speech_pad_samples
    min_silence_samples = sampling_rate * o["min_silence_duration_ms"] / 1000
    min_silence_samples_at_max_speech = sampling_rate * 98 / 1000
    triggered, speeches, cur = False, [], {}
    temp_end = prev_end = next_start = 0
    for i, p in enumerate(probs):
        if p >= threshold and temp_end:
            temp_end = 0
            if next_start < prev_end:
                next_start = ws * i
        if p >= threshold and not triggered:
            triggered = True
            cur["start"] = ws * i
            continue
        if triggered and ws * i - cur["start"] > max_speech_samples:
            if prev_end:
                cur["end"] = prev_end
                speeches.append(cur)
                cur = {}
                if next_start < prev_end:  # reached silence (< neg_threshold) and still not speech
                    triggered = False
                else:
                    cur["start"] = next_start
                prev_end = next_start = temp_end = 0
            else:
                cur["end"] = ws * i
                speeches.append(cur)
                cur = {}
                prev_end = next_start = temp_end = 0
                triggered = False
                continue
        if p < neg_threshold and triggered:
            if not temp_end:
                temp_end = ws * i
            if ws * i - temp_end > min_silence_samples_at_max_speech:
                prev_end = temp_end
            if ws * i - temp_end < min_silence_samples:
                continue
            cur["end"] = temp_end
            if cur["end"] - cur["start"] > min_speech_samples:
                speeches.append(cur)
            cur = {}
            prev_end = next_start = temp_end = 0
            triggered = False
            continue
    if cur and n_samples - cur["start"] > min_speech_samples:
        cur["end"] = n_samples
        speeches.append(cur)
    for i, sp in enumerate(speeches):
        if i == 0:
            sp["start"] = int(max(0, sp["start"] - speech_pad_samples))
        if i != len(speeches) - 1:
            gap = speeches[i + 1]["start"] - sp["end"]
            if gap < 2 * speech_pad_samples:
                sp["end"] += int(gap // 2)
                speeches[i + 1]["start"] = int(max(0, speeches[i + 1]["start"] - gap // 2))
            else:
                sp["end"] = int(min(n_samples, sp["end"] + speech_pad_samples))
                speeches[i + 1]["start"] = int(max(0, speeches[i + 1]["start"] - speech_pad_samples))
        else:
            sp["end"] = int(min(n_samples, sp["end"] + speech_pad_samples))
    return speeches


def collect_chunks(audio, chunks):
    """The speech chunks of `audio` concatenated (faster-whisper collect_chunks without a max duration)."""
    if not chunks:
        return np.zeros(0, np.float32)
    return np.concatenate([np.asarray(audio[c["start"]:c["end"]], np.float32) for c in chunks])


class SpeechTimestampsMap:
    """Time in the concatenated speech -> time in the original audio (faster-whisper vad.SpeechTimestampsMap)."""

    def __init__(self, chunks, sampling_rate: int = SAMPLE_RATE, time_precision: int = 2):
        self.sampling_rate, self.time_precision = sampling_rate, time_precision
        self.chunk_end_sample, self.total_silence_before = [], []
        previous_end = silent = 0
        for c in chunks:
            silent += c["start"] - previous_end
            previous_end = c["end"]
            self.chunk_end_sample.append(c["end"] - silent)
            self.total_silence_before.append(silent / sampling_rate)

    def get_chunk_index(self, time: float, is_end: bool = False) -> int:
        import bisect
        sample = int(time * self.sampling_rate)
        if is_end and sample in self.chunk_end_sample:
            return self.chunk_end_sample.index(sample)
        return min(bisect.bisect(self.chunk_end_sample, sample), len(self.chunk_end_sample) - 1)

    def get_original_time(self, time: float, chunk_index: int | None = None, is_end: bool = False) -> float:
        if chunk_index is None:
            chunk_index = self.get_chunk_index(time, is_end)
        return round(self.total_silence_before[chunk_index] + time, self.time_precision)


def restore_speech_timestamps(segments, chunks, sampling_rate: int = SAMPLE_RATE):
    """faster-whisper restore_speech_timestamps: words mapped through the chunk of their midpoint, segments from
    their words (or their own start / end)."""
    ts = SpeechTimestampsMap(chunks, sampling_rate)
    for seg in segments:
        if seg.words:
            for w in seg.words:
                k = ts.get_chunk_index((w.start + w.end) / 2)
                w.start = ts.get_original_time(w.start, k)
                w.end = ts.get_original_time(w.end, k)
            seg.start, seg.end = seg.words[0].start, seg.words[-1].end
        else:
            seg.start = ts.get_original_time(seg.start)
            seg.end = ts.get_original_time(seg.end, is_end=True)
        yield seg
