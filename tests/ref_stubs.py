"""Deterministic stand-ins for the third-party modules the reference imports but does not vendor:
faster_whisper.WhisperModel, whisper_online.{FasterWhisperASR, OnlineASRProcessor}, torch.hub's Silero model.

Used twice, with the SAME objects, so that a recorded trace means the same thing on both sides:
  * tests/golden/make_ref_plumbing.py drives the reference's own asr_components.py / enhanced_asr_processor.py
    through these stubs (in the build container only) and records every call into ref_plumbing.json;
  * tests/test_ref_plumbing.py drives wmx.asr / wmx.online through the same stubs and compares the traces.
Test infrastructure only: nothing under realtime-whisper-asr_amd/ imports this module.
"""
from __future__ import annotations

import numpy as np

CALLS: list = []  # global call log the recording stubs append to


def _r(x):
    return round(float(x), 6)


def audio_sig(a):
    a = np.asarray(a, np.float64)
    return [int(a.size), _r(a.sum()), _r(np.abs(a).sum())]


class Word:
    def __init__(self, start, end, word, probability=0.9):
        self.start, self.end, self.word, self.probability = start, end, word, probability


class Segment:
    def __init__(self, start, end, words, no_speech_prob=0.01):
        self.start, self.end, self.words, self.no_speech_prob = start, end, words, no_speech_prob
        self.text = "".join(w.word for w in words)


def fake_segments(n_samples, call_no=0, jitter=False):
    """One word per 0.5 s of audio, four words per segment.  Words are a function of their time in the buffer, so
    successive passes over a growing buffer agree on their common prefix; with `jitter` the last word of every
    second call differs (an unstable hypothesis tail, which is what LocalAgreement-n is for)."""
    n = int(n_samples / 16000 / 0.5)
    words = [Word(round(i * 0.5, 2), round(i * 0.5 + 0.4, 2), f" w{i}") for i in range(n)]
    if jitter and words and call_no % 2 == 1:
        words[-1] = Word(words[-1].start, words[-1].end, f" x{len(words) - 1}")
    segs, cur = [], []
    for w in words:
        cur.append(w)
        if len(cur) == 4:
            segs.append(Segment(cur[0].start, cur[-1].end, cur))
            cur = []
    if cur:
        segs.append(Segment(cur[0].start, cur[-1].end, cur))
    return segs


class RecordingWhisperModel:
    """faster_whisper.WhisperModel stub: records the constructor and transcribe keyword arguments."""

    def __init__(self, model_size_or_path, **kwargs):
        CALLS.append(["WhisperModel", model_size_or_path, {k: kwargs[k] for k in sorted(kwargs)}])
        self.n = 0

    def transcribe(self, audio, **kwargs):
        CALLS.append(["transcribe", audio_sig(audio), {k: kwargs[k] for k in sorted(kwargs)}])
        segs = fake_segments(len(audio), self.n)
        self.n += 1
        return iter(segs), {"language": "en"}


class FasterWhisperASRBase:
    """whisper_online.FasterWhisperASR stand-in (the reference subclasses it; every method is overridden)."""
    sep = ""


class RecordingOnline:
    """whisper_online.OnlineASRProcessor stub seen by the VAC gate: records init / insert / process / finish."""
    SAMPLING_RATE = 16000

    def __init__(self, asr=None, tokenizer=None, logfile=None, buffer_trimming=("segment", 15)):
        CALLS.append(["online.__init__", list(buffer_trimming)])
        self.n = 0

    def init(self, offset=None):
        CALLS.append(["online.init", None if offset is None else _r(offset)])

    def insert_audio_chunk(self, audio):
        CALLS.append(["online.insert", audio_sig(audio)])

    def process_iter(self):
        self.n += 1
        CALLS.append(["online.process_iter", self.n])
        return (float(self.n), float(self.n) + 0.5, f"it{self.n}")

    def finish(self):
        self.n += 1
        CALLS.append(["online.finish", self.n])
        return (None, None, f"fin{self.n}")


class ScriptedSilero:
    """torch.hub Silero VAD stand-in: probs[i] is the speech probability of the i-th 512-sample window."""

    def __init__(self, probs):
        self.probs = list(probs)
        self.i = 0

    def reset_states(self):
        self.i = 0

    def __call__(self, x, sr=16000):
        p = self.probs[self.i] if self.i < len(self.probs) else 0.0
        self.i += 1
        return p


class FakeASR:
    """ASR backend for the streaming processors: fake_segments over the buffer it is given; optionally raises on
    the call numbers in `fail_on` (the reset-on-error path of enhanced_asr_processor.py:369-381)."""
    sep = ""

    def __init__(self, jitter=False, fail_on=()):
        self.jitter, self.fail_on, self.n = jitter, set(fail_on), 0
        self.calls = []

    def transcribe(self, audio, init_prompt=""):
        self.n += 1
        self.calls.append([len(audio), init_prompt])
        if self.n in self.fail_on:
            raise RuntimeError(f"scripted failure on call {self.n}")
        return fake_segments(len(audio), self.n, self.jitter)

    def ts_words(self, segments):
        return [(w.start, w.end, w.word) for s in segments for w in s.words]

    def segments_end_ts(self, segments):
        return [s.end for s in segments]


def vad_track(seed=3, n_windows=400):
    """Scripted speech probabilities: speech bursts of 0.5-3 s with gaps of 0.1-1.5 s (so both the hysteresis
    and the min-silence rule fire), values spread over [0, 1]."""
    rng = np.random.default_rng(seed)
    out, speech = [], False
    while len(out) < n_windows:
        n = int(rng.integers(16, 94)) if speech else int(rng.integers(3, 47))
        lo, hi = (0.55, 1.0) if speech else (0.0, 0.45)
        out.extend(float(round(v, 4)) for v in rng.uniform(lo, hi, n))
        speech = not speech
    return out[:n_windows]


def chunk_sizes(seed=4, total=400 * 512):
    rng = np.random.default_rng(seed)
    out, s = [], 0
    choices = [640, 640, 640, 512, 1000, 333, 2048, 160]
    while s < total:
        n = int(choices[int(rng.integers(0, len(choices)))])
        out.append(n)
        s += n
    return out


def audio_stream(seed=5, n=400 * 512):
    rng = np.random.default_rng(seed)
    return (0.1 * rng.standard_normal(n)).astype(np.float32)
