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

from ._lib import WMX_ERR_NUMERIC, WmxError
from .engine import ALIGNMENT_HEADS, Context, Model
from .tokenizer import LANGUAGES, load_tokenizer, suppressed_tokens

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


def add_word_timestamps(subsegments, alignment, seek, last_speech_timestamp, prepended=PREPEND_PUNCT,
                        appended=APPEND_PUNCT):
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
    merge_punctuations(alignment, prepended, appended)
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


# faster-whisper 1.2.1 WhisperModel.transcribe keywords this engine does not implement, with the value that means
# "off"; any other value raises NotImplementedError instead of being silently ignored
_FW_UNSUPPORTED = {
    "prefix": None,
    "hotwords": None,
    "clip_timestamps": "0",
    "hallucination_silence_threshold": None,
    "multilingual": False,
    "repetition_penalty": 1,
    "no_repeat_ngram_size": 0,
    "chunk_length": None,
    "language_detection_segments": 1,
}
# accepted and without effect on this path (faster-whisper semantics preserved)
_FW_NO_EFFECT = ("log_progress", "language_detection_threshold")


def _check_kwargs(kw):
    for k, v in kw.items():
        if k in _FW_UNSUPPORTED:
            off = _FW_UNSUPPORTED[k]
            if v != off and not (k == "chunk_length" and v == 30) and not (k == "clip_timestamps" and v in ([], None)):
                raise NotImplementedError(f"faster-whisper option {k}={v!r} is not implemented by the MI355X engine")
        elif k not in _FW_NO_EFFECT:
            raise TypeError(f"transcribe() got an unexpected keyword argument {k!r}")


def _temperatures(temperature):
    """faster-whisper: a float is a one-entry schedule; a list / tuple is the fallback schedule."""
    ts = [float(t) for t in (temperature if isinstance(temperature, (list, tuple)) else [temperature])]
    if not ts or any(not np.isfinite(t) or t < 0 for t in ts):
        raise ValueError(f"temperature={temperature!r}: expected finite values >= 0")
    return ts


def call_seed(seed: int, call: int, temp_index: int) -> int:
    """The sampling seed of one decode call: splitmix64 of (model seed, call counter, temperature index), low 32 bits."""
    z = (seed * 0x9E3779B97F4A7C15 + (call << 8) + temp_index + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return (z ^ (z >> 31)) & 0xFFFFFFFF


def get_end(segments):
    """faster-whisper get_end: the last word's end, else the last segment's end."""
    return next((w["end"] for s in reversed(segments) for w in reversed(s.get("words") or [])),
                segments[-1]["end"] if segments else None)


class WhisperModel:
    """MI355X stand-in for faster_whisper.WhisperModel (same constructor keywords the reference passes at
    asr_components.py:244-262; `download_root`/`num_workers` are accepted and ignored — weights are either a
    local HF/openai-named checkpoint (safetensors) or the build-owned synthetic initialisation)."""

    def __init__(self, model_size_or_path="large-v3", device="cuda", device_index=0, compute_type="float16",
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
        self.device_index = int(device_index)
        self.model = Model(name, int(device_index), compute_type)
        self.dims = self.model.dims
        self.tokenizer = load_tokenizer(model_dir, self.dims.n_vocab)
        if model_dir:
            _load_checkpoint(self.model, model_dir)
        else:
            self.model.init_synthetic(seed)
        self.name = name
        # a checkpoint's own alignment heads win over the per-size table (CT2 keeps them in config.json, HF in
        # generation_config.json; fine-tuned / distilled models differ from openai's table)
        self.alignment_heads = _checkpoint_alignment_heads(model_dir) or ALIGNMENT_HEADS.get(name)
        self.max_batch = max_batch
        self.default_beam = beam_size
        self.max_new_tokens = max_new_tokens
        self.suppress_tokens = [-1] if suppress_tokens is None else list(suppress_tokens)
        self.use_graph = use_graph
        # sampling (T > 0): every decode call draws with its own seed, mixed from the model seed, a per-model call
        # counter and the temperature's index in the fallback schedule (faster-whisper / CT2 draw fresh randomness per
        # generate call, so a T = 0.4 retry after a failed T = 0.2 attempt is not correlated with it); the same model
        # seed and call sequence replays the same draws
        self.sample_seed = seed
        self._sample_calls = 0
        self._ctx = {}
        # transcribe_batch: split a batch of >= `groups` windows over that many contexts decoding concurrently in step
        # (wmx_ctx_set_lockstep, as bench.py's two groups; 1 = one context per batch)
        self.groups = 1
        # what the calls cost on the device (bench.py's latency lines decompose a call with it): decoded windows
        # (engine transcribe rows, fallback retries included), engine calls, decode steps those calls ran
        self.counters = {"windows": 0, "engine_calls": 0, "decode_steps": 0}

    def context(self, beam_size, language_token, task, word_timestamps, without_timestamps=False, patience=1.0,
                length_penalty=1.0, suppress_blank=True, suppress_tokens=None, max_initial_timestamp=1.0,
                max_new_tokens=None, temperature=0.0, best_of=5, group=None):
        sup = tuple(suppressed_tokens(self.tokenizer.sp, self.suppress_tokens if suppress_tokens is None
                                      else suppress_tokens))
        mit = None if max_initial_timestamp is None else int(round(max_initial_timestamp / TIME_PRECISION))
        mnt = max_new_tokens or self.max_new_tokens or 448
        temperature = float(temperature)
        best_of = int(best_of) if temperature > 0 else 5
        key = (beam_size, language_token, task, word_timestamps, without_timestamps, float(patience),
               float(length_penalty), bool(suppress_blank), sup, mit, mnt, temperature, best_of)
        opts = key
        if group is not None:  # (g, n): member g of n contexts that decode one batch concurrently, in step
            key = key + (group,)
        if key not in self._ctx:
            ctx = Context(self.model, max_batch=self.max_batch, beam_size=beam_size, patience=patience,
                          length_penalty=length_penalty, max_new_tokens=mnt, task=task, language=language_token,
                          without_timestamps=without_timestamps, max_initial_timestamp_index=mit,
                          suppress_blank=suppress_blank, suppress_tokens=sup, word_timestamps=word_timestamps,
                          alignment_heads=self.alignment_heads, use_graph=self.use_graph,
                          max_audio_samples=2 * 480000, temperature=temperature, best_of=best_of,
                          sample_seed=self.sample_seed)
            if group is not None:  # one lockstep key per (model, options, group count)
                ctx.set_lockstep(1 + (hash((id(self), opts, group[1])) & 0x3FFFFFFF), group[1])
            self._ctx[key] = ctx
        return self._ctx[key]

    # ---- faster-whisper WhisperModel.transcribe ----
    def transcribe(self, audio, language=None, task="transcribe", beam_size=5, best_of=5, patience=1.0,
                   length_penalty=1.0, temperature=0.0, initial_prompt=None, word_timestamps=False,
                   condition_on_previous_text=True, no_speech_threshold=0.6, log_prob_threshold=-1.0,
                   compression_ratio_threshold=2.4, without_timestamps=False, suppress_blank=True,
                   suppress_tokens=(-1,), max_initial_timestamp=1.0, max_new_tokens=None,
                   prepend_punctuations=PREPEND_PUNCT, append_punctuations=APPEND_PUNCT,
                   prompt_reset_on_temperature=0.5, vad_filter=False, vad_parameters=None, **kwargs):
        """faster-whisper 1.2.1 transcribe + generate_segments over 30 s windows (seek loop).  Language detection
        runs once, on the first window, and every later window decodes with that language; with word timestamps
        a window that does not end on a single timestamp moves seek to its last word's end (round(end * 100))."""
        _check_kwargs(kwargs)
        temps = _temperatures(temperature)
        audio = np.asarray(audio, dtype=np.float32)
        duration = len(audio) / SAMPLE_RATE
        speech_chunks = None
        if vad_filter:  # faster-whisper: transcribe only the speech chunks, map the times back afterwards
            from .vad import collect_chunks, get_speech_timestamps, speech_probs
            params = dict(vars(vad_parameters)) if hasattr(vad_parameters, "__dict__") else dict(vad_parameters or {})
            speech_chunks = get_speech_timestamps(speech_probs(self.vad_engine(), audio), len(audio), **params)
            audio = collect_chunks(audio, speech_chunks)
        tok = self.tokenizer
        sp = tok.sp
        lang_tok = None if language is None else sp.language_token(language)
        ctx_kw = dict(without_timestamps=without_timestamps, patience=patience, length_penalty=length_penalty,
                      suppress_blank=suppress_blank, suppress_tokens=list(suppress_tokens or []),
                      max_initial_timestamp=max_initial_timestamp, max_new_tokens=max_new_tokens)
        all_tokens = []
        prompt_reset_since = 0
        if initial_prompt is not None:
            if isinstance(initial_prompt, str):
                all_tokens.extend(tok.encode(" " + initial_prompt.strip()))
            else:
                all_tokens.extend(initial_prompt)
        content_frames = len(audio) // HOP
        seek = 0
        segments, last_speech = [], 0.0
        detected, det_prob = language, 1.0
        punct = (prepend_punctuations, append_punctuations)
        while seek < content_frames:
            segment_size = min(N_FRAMES, content_frames - seek)
            prompt = all_tokens[prompt_reset_since:] if condition_on_previous_text else []
            r, used_t = self._decode_with_fallback(audio, seek, prompt, temps, beam_size, best_of, lang_tok, task,
                                                   word_timestamps, ctx_kw, compression_ratio_threshold,
                                                   log_prob_threshold, no_speech_threshold)
            if detected is None:
                detected, det_prob = sp.language_code(r.language), r.language_prob
            if lang_tok is None:
                lang_tok = sp.lang0 + LANGUAGES.index(detected)  # detected once, fixed for later windows
            segs, toks, seek_new, last_speech = self._window_segments(
                r, seek, segment_size, word_timestamps, detected, last_speech, len(segments),
                no_speech_threshold, log_prob_threshold, punct)
            segments.extend(segs)
            all_tokens.extend(toks)
            if not condition_on_previous_text or used_t > prompt_reset_on_temperature:
                prompt_reset_since = len(all_tokens)
            seek = seek_new if seek_new > seek else seek + max(1, segment_size)
        if speech_chunks:
            from .vad import restore_speech_timestamps
            segments = list(restore_speech_timestamps(segments, speech_chunks))
        info = TranscriptionInfo(detected or "en", det_prob, duration, len(audio) / SAMPLE_RATE)
        return iter(segments), info

    def vad_engine(self):
        """The Silero network of vad_filter (device, one slot): weights from the safetensors file named by
        WMX_SILERO_WEIGHTS when set, else synthetic (no Silero checkpoint ships in this image)."""
        if getattr(self, "_vad", None) is None:
            import os

            from .vad import SileroVADEngine, load_state_dict
            path = os.environ.get("WMX_SILERO_WEIGHTS")
            self._vad = SileroVADEngine(load_state_dict(path) if path else None, device=self.device_index,
                                        max_streams=1, max_windows=64)
        return self._vad

    def _count(self, ctx, windows):
        # (host tests build the model without __init__ and drive it with engine stand-ins)
        c = self.__dict__.setdefault("counters", {"windows": 0, "engine_calls": 0, "decode_steps": 0})
        c["windows"] += windows
        c["engine_calls"] += 1
        steps = getattr(ctx, "last_steps", None)
        c["decode_steps"] += steps() if steps else 0

    def _decode_with_fallback(self, audio, seek, prompt, temps, beam_size, best_of, lang_tok, task, word_timestamps,
                              ctx_kw, compression_ratio_threshold, log_prob_threshold, no_speech_threshold):
        """faster-whisper generate_with_fallback: decode at each temperature of the schedule until the result passes
        the compression-ratio and log-prob checks (a likely-silent window passes); if none does, keep the best
        avg_logprob among those under the compression threshold (else among all), reported at the last
        temperature.  T = 0: beam search (beam_size); T > 0: best_of sampled rows."""
        results = []
        for ti, t in enumerate(temps):
            ctx = self.context(beam_size, lang_tok, task, word_timestamps, temperature=t, best_of=best_of, **ctx_kw)
            if t > 0:
                ctx.set_sample_seed(call_seed(self.sample_seed, self._sample_calls, ti))
                self._sample_calls += 1
            # the window's features come from the whole buffer (global max normalisation) -> pass the full audio
            r = ctx.transcribe([audio], prompts=[prompt], seek=[seek])[0]
            self._count(ctx, 1)
            cr = compression_ratio(self.tokenizer.decode([x for x in r.tokens if x < self.tokenizer.sp.eot]).strip())
            results.append((r, cr))
            needs = False
            if compression_ratio_threshold is not None and cr > compression_ratio_threshold:
                needs = True
            if log_prob_threshold is not None and r.avg_logprob < log_prob_threshold:
                needs = True
            if (no_speech_threshold is not None and r.no_speech_prob > no_speech_threshold
                    and log_prob_threshold is not None and r.avg_logprob < log_prob_threshold):
                needs = False  # silence
            if not needs:
                return r, t
        below = [x for x in results if compression_ratio_threshold is None or x[1] <= compression_ratio_threshold]
        return max(below or results, key=lambda x: x[0].avg_logprob)[0], temps[-1]

    def _window_segments(self, r, seek, segment_size, word_timestamps, language, last_speech, first_id,
                         no_speech_threshold=0.6, log_prob_threshold=-1.0, punct=(PREPEND_PUNCT, APPEND_PUNCT)):
        """faster-whisper generate_segments body for one decoded window -> (segments, tokens, seek, last_speech)."""
        tok, sp = self.tokenizer, self.tokenizer.sp
        time_offset = seek * HOP / SAMPLE_RATE
        segment_duration = segment_size * HOP / SAMPLE_RATE
        if no_speech_threshold is not None:
            skip = r.no_speech_prob > no_speech_threshold
            if log_prob_threshold is not None and r.avg_logprob > log_prob_threshold:
                skip = False  # high enough log prob despite the no-speech probability
            if skip:
                return [], [], seek + segment_size, last_speech
        subs, seek_new, single_ending = split_segments_by_timestamps(
            sp.timestamp_begin, list(r.tokens), time_offset, segment_size, segment_duration, seek)
        if word_timestamps:
            text_tokens = [t for t in r.tokens if t < sp.eot]
            alignment = words_from_jumps(tok, text_tokens, r.jump_times, r.text_token_probs, language or "en")
            last_speech = add_word_timestamps(subs, alignment, seek, last_speech, *punct)
            if not single_ending:
                last_word_end = get_end(subs)
                if last_word_end is not None and last_word_end > time_offset:
                    seek_new = round(last_word_end * (SAMPLE_RATE // HOP))
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

    def _transcribe_groups(self, G, chunk, pr, beam, lang_tok, task, word_timestamps, best_of):
        """One batch split over G contexts, each on its own host thread (ctypes drops the GIL inside libwmx), their
        decode loops started together and kept in step (wmx_ctx_set_lockstep): each layer's weights are then read once
        for all groups, and one group's kernel boundaries overlap the others' work -- the bench's two-group form."""
        from concurrent.futures import ThreadPoolExecutor
        parts = [p for p in np.array_split(np.arange(len(chunk)), G) if len(p)]
        ctxs = [self.context(beam, lang_tok, task, word_timestamps, temperature=0.0, best_of=best_of, group=(g, G))
                for g in range(len(parts))]
        pool = self.__dict__.get("_group_pool")
        if pool is None or pool._max_workers < G:  # (groups raised since: one thread per lockstep member)
            if pool is not None:
                pool.shutdown(wait=True)
            pool = self._group_pool = ThreadPoolExecutor(max_workers=G)
        futs = [pool.submit(c.transcribe, [chunk[j] for j in p], prompts=[pr[j] for j in p])
                for c, p in zip(ctxs, parts)]
        from concurrent.futures import wait
        wait(futs)  # every group finishes before any error propagates (a context serves one call at a time)
        res = [f.result() for f in futs]  # (raises before any group is counted: the fallback re-runs the batch)
        for c, p in zip(ctxs, parts):
            self._count(c, len(p))
        return [r for part in res for r in part]

    def _transcribe_isolating(self, ctx, idx, chunk, pr, out):
        """ctx.transcribe of a batch; a WMX_ERR_NUMERIC naming one window (one stream's non-finite decode, e.g. NaN
        samples from one microphone) fails that stream only: its error goes to out[idx[k]] and the batch is re-run
        without it (the reference runs each stream on its own).  Returns the results of the windows kept,
        in order; out[] of the failed ones is set."""
        import re
        live = list(range(len(idx)))
        while live:
            try:
                res = ctx.transcribe([chunk[k] for k in live], prompts=[pr[k] for k in live])
                self._count(ctx, len(live))
                full = [None] * len(idx)
                for k, r in zip(live, res):
                    full[k] = r
                return [r for r in full if r is not None]
            except WmxError as e:
                m = re.search(r"window (\d+)", str(e))
                if e.status != WMX_ERR_NUMERIC or not m or int(m.group(1)) >= len(live):
                    raise
                bad = live.pop(int(m.group(1)))
                out[idx[bad]] = e
        return []

    def transcribe_batch(self, audios, prompts=None, language=None, task="transcribe", beam_size=None,
                         word_timestamps=True, no_speech_threshold=0.6, log_prob_threshold=-1.0, temperature=0.0,
                         best_of=5):
        """Many independent streams' buffers in ONE libwmx launch sequence (one window each).  prompts: per-stream
        previous text (str) or token lists.  Buffers longer than one 30 s window (a streaming buffer nothing has
        committed from yet) go through the full seek loop of transcribe() instead.  Returns per stream a list of
        segments, or the exception that stream's call raised (the caller decides, per stream, what to do)."""
        tok, sp = self.tokenizer, self.tokenizer.sp
        beam = beam_size or self.default_beam
        lang_tok = None if language is None else sp.language_token(language)
        prompts = list(prompts) if prompts is not None else [None] * len(audios)
        out = [None] * len(audios)
        short = []
        temps = _temperatures(temperature)
        for i, a in enumerate(audios):
            if len(a) > N_FRAMES * HOP or len(temps) > 1:  # several windows, or a fallback schedule: per stream
                p = prompts[i]
                try:
                    segs, _ = self.transcribe(a, language=language, task=task, beam_size=beam, best_of=best_of,
                                              temperature=temps, initial_prompt=p,
                                              word_timestamps=word_timestamps,
                                              no_speech_threshold=no_speech_threshold,
                                              log_prob_threshold=log_prob_threshold)
                    out[i] = list(segs)
                except Exception as e:  # per stream, like EnhancedOnlineASRProcessor.process_iter
                    out[i] = e
            else:
                short.append(i)
        ctx = self.context(beam, lang_tok, task, word_timestamps, temperature=temps[0], best_of=best_of)
        for b0 in range(0, len(short), self.max_batch):
            if temps[0] > 0:  # fresh draws per call (call_seed)
                ctx.set_sample_seed(call_seed(self.sample_seed, self._sample_calls, 0))
                self._sample_calls += 1
            idx = short[b0: b0 + self.max_batch]
            chunk = [np.asarray(audios[i], np.float32) for i in idx]
            pr = []
            for i in idx:
                p = prompts[i]
                if isinstance(p, str):
                    pr.append(tok.encode(" " + p.strip()))
                else:
                    pr.append(list(p or []))
            G = max(1, int(getattr(self, "groups", 1)))
            try:
                if G > 1 and temps[0] == 0 and len(idx) >= G:
                    try:
                        res = self._transcribe_groups(G, chunk, pr, beam, lang_tok, task, word_timestamps, best_of)
                    except WmxError as e:
                        if e.status != WMX_ERR_NUMERIC:
                            raise
                        # a non-finite window in one group: the one-context path below isolates it
                        res = self._transcribe_isolating(ctx, idx, chunk, pr, out)
                else:
                    res = self._transcribe_isolating(ctx, idx, chunk, pr, out)
            except Exception as e:
                for i in idx:
                    if out[i] is None:
                        out[i] = e
                continue
            keep = [k for k, i in enumerate(idx) if out[i] is None]  # (windows that failed alone already hold it)
            idx, chunk = [idx[k] for k in keep], [chunk[k] for k in keep]
            for i, a, r in zip(idx, chunk, res):
                lang = language or sp.language_code(r.language)
                segs, _, _, _ = self._window_segments(r, 0, min(N_FRAMES, len(a) // HOP), word_timestamps, lang,
                                                      0.0, 0, no_speech_threshold, log_prob_threshold)
                out[i] = segs
        return out


def _checkpoint_alignment_heads(model_dir):
    """[[layer, head], ...] from a model directory's config.json (CTranslate2) or generation_config.json (HF)."""
    import json
    import os
    if not model_dir:
        return None
    for f in ("config.json", "generation_config.json"):
        p = os.path.join(model_dir, f)
        if os.path.exists(p):
            heads = json.load(open(p)).get("alignment_heads")
            if heads:
                return [tuple(int(x) for x in h) for h in heads]
    return None


def _infer_name(model_dir):
    import json
    import os
    if os.path.exists(os.path.join(model_dir, "model.bin")):  # CTranslate2 directory (the reference's models_fast/)
        from .ct2 import ct2_dims, read_model_bin
        dims = ct2_dims(read_model_bin(os.path.join(model_dir, "model.bin"))[2])
        cfg = {"d_model": dims["n_audio_state"], "decoder_layers": dims["n_text_layer"], "num_mel_bins": dims["n_mels"]}
    else:
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
    """A CTranslate2 model.bin (wmx.ct2: f32 / f16 / bf16 / int8 storage) or HF Whisper safetensors (any of f32 / f16 /
    bf16 storage) -> wmx_model_set_tensor (rounds to the model dtype, packs the decoder projections).  bf16 has no
    numpy dtype, so safetensors are read through torch."""
    import glob
    import os
    if os.path.exists(os.path.join(model_dir, "model.bin")):  # CTranslate2 (faster-whisper) directory
        from .ct2 import load_ct2_dir
        scales = {}  # (an int8 model keeps an int8 checkpoint's own grid: its q and row scales)
        model.load_state_dict(load_ct2_dir(model_dir, scales)[1], row_scales=scales)
        return
    files = sorted(glob.glob(os.path.join(model_dir, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no model.bin (CTranslate2) or *.safetensors (HF) in {model_dir}")
    from safetensors.torch import load_file
    sd = {}
    for f in files:
        for k, v in load_file(f).items():
            sd[k] = v.float().numpy()
    model.load_state_dict(sd)
