"""faster-whisper `WhisperModel.transcribe` semantics on top of libwmx (host-side, per window).

Restated from faster-whisper 1.2.1 transcribe.py (not in the container): the caller in the
reference is asr_components.py:279-288 with beam_size=5, temperature=0.0, word_timestamps=True,
condition_on_previous_text=True.  The numeric work (log-mel, encoder, decode, alignment, DTW) is one
wmx_transcribe call per 30 s window; this module keeps faster-whisper's window loop, prompt bookkeeping,
timestamp-based segment splitting, no-speech skip and word-timestamp post-processing.
"""
from __future__ import annotations

import itertools
import math
import zlib
from dataclasses import dataclass, field

import numpy as np

from .engine import ALIGNMENT_HEADS, Context, Model
from .tokenizer import DEFAULT_SUPPRESS, LANGUAGES, load_tokenizer

SAMPLE_RATE = 16000
HOP = 160
N_FRAMES = 3000
TIME_PRECISION = 0.02
INPUT_STRIDE = 2
PREPEND_PUNCT = "\"'“¿([{-"
APPEND_PUNCT = "\"'.。,，!！?？:：”)]}、"


@dataclass
class Word:
    start: float
    end: float
    word: str
    probability: float

    def _asdict(self):
        return {"start": self.start, "end": self.end, "word": self.word, "probability": self.probability}


@dataclass
class Segment:
    id: int
    seek: int
    start: float
    end: float
    text: str
    tokens: list
    avg_logprob: float
    compression_ratio: float
    no_speech_prob: float
    words: list | None
    temperature: float = 0.0


@dataclass
class TranscriptionInfo:
    language: str
    language_probability: float
    duration: float
    duration_after_vad: float
    all_language_probs: list | None = None
    transcription_options: dict = field(default_factory=dict)


def compression_ratio(text: str) -> float:
    b = text.encode("utf-8")
    return len(b) / max(1, len(zlib.compress(b)))


def split_segments_by_timestamps(tb, tokens, time_offset, segment_size, segment_duration, seek):
    """faster-whisper WhisperModel._split_segments_by_timestamps."""
    segs = []
    single_ending = len(tokens) >= 2 and tokens[-2] < tb <= tokens[-1]
    consecutive = [i for i in range(len(tokens)) if i > 0 and tokens[i] >= tb and tokens[i - 1] >= tb]
    if consecutive:
        slices = list(consecutive)
        if single_ending:
            slices.append(len(tokens))
        last = 0
        for cur in slices:
            st = tokens[last:cur]
            segs.append(dict(seek=seek, start=time_offset + (st[0] - tb) * TIME_PRECISION,
                             end=time_offset + (st[-1] - tb) * TIME_PRECISION, tokens=st))
            last = cur
        if single_ending:
            seek += segment_size
        else:
            seek += (tokens[last - 1] - tb) * INPUT_STRIDE
    else:
        duration = segment_duration
        ts = [t for t in tokens if t >= tb]
        if ts and ts[-1] != tb:
            duration = (ts[-1] - tb) * TIME_PRECISION
        segs.append(dict(seek=seek, start=time_offset, end=time_offset + duration, tokens=tokens))
        seek += segment_size
    return segs, seek, single_ending


def merge_punctuations(alignment, prepended, appended):
    """openai timing.merge_punctuations (faster-whisper identical)."""
    i, j = len(alignment) - 2, len(alignment) - 1
    while i >= 0:
        prev, foll = alignment[i], alignment[j]
        if prev["word"].startswith(" ") and prev["word"].strip() in prepended:
            foll["word"] = prev["word"] + foll["word"]
            foll["tokens"] = prev["tokens"] + foll["tokens"]
            prev["word"], prev["tokens"] = "", []
        else:
            j = i
        i -= 1
    i, j = 0, 1
    while j < len(alignment):
        prev, foll = alignment[i], alignment[j]
        if not prev["word"].endswith(" ") and foll["word"] in appended:
            prev["word"] = prev["word"] + foll["word"]
            prev["tokens"] = prev["tokens"] + foll["tokens"]
            foll["word"], foll["tokens"] = "", []
        else:
            i = j
        j += 1


def words_from_jumps(tokenizer, text_tokens, jump_times, token_probs, language):
    """faster-whisper find_alignment post-processing: word grouping + start/end from DTW jump times."""
    words, word_tokens = tokenizer.split_to_word_tokens(list(text_tokens) + [tokenizer.eot], language)
    if len(word_tokens) <= 1 or jump_times is None:
        return []
    bounds = np.pad(np.cumsum([len(t) for t in word_tokens[:-1]]), (1, 0))
    if len(bounds) <= 1:
        return []
    jt = np.asarray(jump_times)
    starts, ends = jt[bounds[:-1]], jt[bounds[1:]]
    probs = np.asarray(token_probs if token_probs is not None else np.ones(len(text_tokens)))
    wp = [float(np.mean(probs[i:j])) if j > i else 0.0 for i, j in zip(bounds[:-1], bounds[1:])]
    return [dict(word=w, tokens=t, start=float(s), end=float(e), probability=p)
            for w, t, s, e, p in zip(words, word_tokens, starts, ends, wp)]


def add_word_timestamps(subsegments, alignment, seek, last_speech_timestamp):
    """faster-whisper add_word_timestamps for one window (median-duration clamps, punctuation merge,
    segment-boundary fixes)."""
    durs = np.array([w["end"] - w["start"] for w in alignment])
    durs = durs[durs.nonzero()]
    median = min(0.7, float(np.median(durs))) if len(durs) else 0.0
    max_dur = median * 2
    if len(durs):
        marks = ".。!！?？"
        for i in range(1, len(alignment)):
            if alignment[i]["end"] - alignment[i]["start"] > max_dur:
                if alignment[i]["word"] in marks:
                    alignment[i]["end"] = alignment[i]["start"] + max_dur
                elif alignment[i - 1]["word"] in marks:
                    alignment[i]["start"] = alignment[i]["end"] - max_dur
    merge_punctuations(alignment, PREPEND_PUNCT, APPEND_PUNCT)
    time_offset = seek * HOP / SAMPLE_RATE
    wi = 0
    for sub in subsegments:
        saved, words = 0, []
        ntext = len([t for t in sub["tokens"] if t < 50257])
        while wi < len(alignment) and saved < ntext:
            tm = alignment[wi]
            if tm["word"]:
                words.append(dict(word=tm["word"], start=round(time_offset + tm["start"], 2),
                                  end=round(time_offset + tm["end"], 2), probability=tm["probability"]))
            saved += len(tm["tokens"])
            wi += 1
        if words:
            if words[0]["end"] - last_speech_timestamp > median * 4 and (
                    words[0]["end"] - words[0]["start"] > max_dur
                    or (len(words) > 1 and words[1]["end"] - words[0]["start"] > max_dur * 2)):
                if len(words) > 1 and words[1]["end"] - words[1]["start"] > max_dur:
                    boundary = max(words[1]["end"] / 2, words[1]["end"] - max_dur)
                    words[0]["end"] = words[1]["start"] = boundary
                words[0]["start"] = max(0, words[0]["end"] - max_dur)
            if sub["start"] < words[0]["end"] and sub["start"] - 0.5 > words[0]["start"]:
                words[0]["start"] = max(0, min(words[0]["end"] - median, sub["start"]))
            else:
                sub["start"] = words[0]["start"]
            if sub["end"] > words[-1]["start"] and sub["end"] + 0.5 < words[-1]["end"]:
                words[-1]["end"] = max(words[-1]["start"] + median, sub["end"])
            else:
                sub["end"] = words[-1]["end"]
            last_speech_timestamp = sub["end"]
        sub["words"] = words
    return last_speech_timestamp


class WhisperModel:
    """MI355X stand-in for faster_whisper.WhisperModel (same constructor keywords the reference passes at
    asr_components.py:251-264; `download_root`/`num_workers` are accepted and ignored — weights are either a
    local HF/openai-named checkpoint (safetensors) or the build-owned synthetic initialisation)."""

    def __init__(self, model_size_or_path="large-v3", device="cuda", device_index=0, compute_type="bfloat16",
                 cpu_threads=0, num_workers=1, download_root=None, local_files_only=True, seed=1, max_batch=1,
                 beam_size=5, max_new_tokens=None, suppress_tokens=None, use_graph=True):
        if device not in ("cuda", "auto", "gpu", "rocm"):
            raise ValueError("wmx runs on MI355X only (device='cuda'); there is no CPU path")
        if isinstance(device_index, (list, tuple)):
            device_index = device_index[0]
        name = model_size_or_path
        model_dir = None
        import os
        if isinstance(name, str) and os.path.isdir(name):
            model_dir = name
            name = _infer_name(model_dir)
        self.model = Model(name, int(device_index), compute_type)
        self.dims = self.model.dims
        self.tokenizer = load_tokenizer(model_dir, self.dims.n_vocab)
        if model_dir:
            _load_checkpoint(self.model, model_dir)
        else:
            self.model.init_synthetic(seed)
        self.name = name
        self.max_batch = max_batch
        self.default_beam = beam_size
        self.max_new_tokens = max_new_tokens
        self.suppress = DEFAULT_SUPPRESS if suppress_tokens is None else list(suppress_tokens)
        self.use_graph = use_graph
        self._ctx = {}

    def context(self, beam_size, language_token, task, word_timestamps, without_timestamps=False):
        key = (beam_size, language_token, task, word_timestamps, without_timestamps)
        if key not in self._ctx:
            self._ctx[key] = Context(self.model, max_batch=self.max_batch, beam_size=beam_size,
                                     max_new_tokens=self.max_new_tokens or 448, task=task, language=language_token,
                                     without_timestamps=without_timestamps, suppress_tokens=self.suppress,
                                     word_timestamps=word_timestamps, alignment_heads=ALIGNMENT_HEADS.get(self.name),
                                     use_graph=self.use_graph, max_audio_samples=2 * 480000)
        return self._ctx[key]

    # ---- faster-whisper WhisperModel.transcribe ----
    def transcribe(self, audio, language=None, task="transcribe", beam_size=5, best_of=5, patience=1.0,
                   length_penalty=1.0, temperature=0.0, initial_prompt=None, word_timestamps=False,
                   condition_on_previous_text=True, no_speech_threshold=0.6, log_prob_threshold=-1.0,
                   compression_ratio_threshold=2.4, without_timestamps=False, vad_filter=False, **_unused):
        audio = np.asarray(audio, dtype=np.float32)
        tok = self.tokenizer
        sp = tok.sp
        lang_tok = None if language is None else sp.language_token(language)
        ctx = self.context(beam_size, lang_tok, task, word_timestamps, without_timestamps)
        all_tokens = []
        prompt_reset_since = 0
        if initial_prompt:
            if isinstance(initial_prompt, str):
                all_tokens.extend(tok.encode(" " + initial_prompt.strip()))
            else:
                all_tokens.extend(initial_prompt)
        content_frames = len(audio) // HOP
        seek = 0
        segments, last_speech = [], 0.0
        detected, det_prob = language, 1.0
        while seek < content_frames:
            segment_size = min(N_FRAMES, content_frames - seek)
            prompt = all_tokens[prompt_reset_since:] if condition_on_previous_text else []
            # the window's features come from the whole buffer (global max normalisation) -> pass the full audio
            r = ctx.transcribe([audio], prompts=[prompt], seek=[seek])[0]
            if detected is None:
                detected, det_prob = sp.language_code(r.language), r.language_prob
            segs, toks, seek_new, last_speech = self._window_segments(
                r, seek, segment_size, word_timestamps, detected, last_speech, len(segments),
                no_speech_threshold, log_prob_threshold)
            segments.extend(segs)
            all_tokens.extend(toks)
            seek = seek_new if seek_new > seek else seek + max(1, segment_size)
        info = TranscriptionInfo(detected or "en", det_prob, len(audio) / SAMPLE_RATE, len(audio) / SAMPLE_RATE)
        return iter(segments), info

    def _window_segments(self, r, seek, segment_size, word_timestamps, language, last_speech, first_id,
                         no_speech_threshold=0.6, log_prob_threshold=-1.0):
        """faster-whisper generate_segments body for one decoded window -> (segments, tokens, seek, last_speech)."""
        tok, sp = self.tokenizer, self.tokenizer.sp
        time_offset = seek * HOP / SAMPLE_RATE
        segment_duration = segment_size * HOP / SAMPLE_RATE
        if no_speech_threshold is not None and r.no_speech_prob > no_speech_threshold and (
                log_prob_threshold is None or r.avg_logprob < log_prob_threshold):
            return [], [], seek + segment_size, last_speech
        subs, seek_new, _ = split_segments_by_timestamps(sp.timestamp_begin, list(r.tokens), time_offset,
                                                         segment_size, segment_duration, seek)
        if word_timestamps:
            text_tokens = [t for t in r.tokens if t < sp.eot]
            alignment = words_from_jumps(tok, text_tokens, r.jump_times, r.text_token_probs, language or "en")
            last_speech = add_word_timestamps(subs, alignment, seek, last_speech)
        out, toks = [], []
        for s in subs:
            text = tok.decode(s["tokens"])
            if s["start"] == s["end"] or not text.strip():
                continue
            words = ([Word(w["start"], w["end"], w["word"], w["probability"]) for w in s.get("words", [])]
                     if word_timestamps else None)
            out.append(Segment(first_id + len(out), seek, s["start"], s["end"], text, s["tokens"], r.avg_logprob,
                               compression_ratio(text), r.no_speech_prob, words))
            toks.extend(s["tokens"])
        return out, toks, seek_new, last_speech

    def transcribe_batch(self, audios, prompts=None, language=None, task="transcribe", beam_size=None,
                         word_timestamps=True, no_speech_threshold=0.6, log_prob_threshold=-1.0):
        """Many independent streams' buffers (each <= 30 s, one window) in ONE libwmx launch sequence.
        prompts: per-stream previous text (str) or token lists.  Returns a list of segment lists."""
        tok, sp = self.tokenizer, self.tokenizer.sp
        beam = beam_size or self.default_beam
        lang_tok = None if language is None else sp.language_token(language)
        ctx = self.context(beam, lang_tok, task, word_timestamps)
        out = []
        for b0 in range(0, len(audios), self.max_batch):
            chunk = [np.asarray(a, np.float32) for a in audios[b0: b0 + self.max_batch]]
            pr = []
            for p in (prompts or [None] * len(audios))[b0: b0 + self.max_batch]:
                if isinstance(p, str):
                    pr.append(tok.encode(" " + p.strip()) if p.strip() else [])
                else:
                    pr.append(list(p or []))
            res = ctx.transcribe(chunk, prompts=pr)
            for a, r in zip(chunk, res):
                lang = language or sp.language_code(r.language)
                segs, _, _, _ = self._window_segments(r, 0, min(N_FRAMES, len(a) // HOP), word_timestamps, lang,
                                                      0.0, 0, no_speech_threshold, log_prob_threshold)
                out.append(segs)
        return out


def _infer_name(model_dir):
    import json
    import os
    cfg = json.load(open(os.path.join(model_dir, "config.json")))
    nm = {80: "large-v2", 128: "large-v3"}
    d = cfg.get("d_model")
    for k, v in {"tiny": 384, "base": 512, "small": 768, "medium": 1024}.items():
        if d == v:
            return k
    if cfg.get("decoder_layers") == 4:
        return "large-v3-turbo"
    return nm.get(cfg.get("num_mel_bins"), "large-v3")


def _load_checkpoint(model, model_dir):
    import glob
    import os
    files = sorted(glob.glob(os.path.join(model_dir, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {model_dir} (CT2 model.bin conversion is not supported yet)")
    from safetensors.numpy import load_file
    sd = {}
    for f in files:
        sd.update(load_file(f))
    model.load_state_dict({k: v.astype(np.float32) for k, v in sd.items()})
