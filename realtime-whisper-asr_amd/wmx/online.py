"""Streaming caller of the hot path, restated in the build's own Python.

* HypothesisBuffer / OnlineASRProcessor / VACOnlineASRProcessor: ufal whisper_streaming whisper_online.py
  (un-vendored in the reference, .gitignore:80) — LocalAgreement-2, prompt = 200-char suffix of committed text
  scrolled out of the buffer, segment trimming.
* VADIterator: silero_vad_iterator.py state machine (threshold, threshold-0.15 hysteresis, min_silence_samples,
  speech_pad_samples).  The Silero network itself is remote-only (torch.hub); the speech probability comes from
  a pluggable model (EnergyVAD default, ScriptedVAD for deterministic tests).
* EnhancedHypothesisBuffer / DynamicBufferManager / EnhancedOnlineASRProcessor / EnhancedVACOnlineASRProcessor /
  DynamicVADIterator / DynamicVACOnlineASRProcessor: the reference's own extensions
  (enhanced_asr_processor.py:32-502, asr_components.py:12-179), same rules.
* StreamBatcher: many independent streams' process_iter() calls served by ONE batched wmx transcribe (the
  MI355X throughput path; streams are independent, so this is pure data parallelism).
"""
from __future__ import annotations

import logging
import sys

import numpy as np

logger = logging.getLogger("wmx.online")
SAMPLING_RATE = 16000


# ------------------------------------------------------------------------------------------------
# whisper_online.HypothesisBuffer (LocalAgreement-2)
# ------------------------------------------------------------------------------------------------
class HypothesisBuffer:
    def __init__(self, logfile=sys.stderr):
        self.commited_in_buffer = []
        self.buffer = []
        self.new = []
        self.last_commited_time = 0
        self.last_commited_word = None
        self.logfile = logfile

    def insert(self, new, offset):
        new = [(a + offset, b + offset, t) for a, b, t in new]
        self.new = [(a, b, t) for a, b, t in new if a > self.last_commited_time - 0.1]
        if len(self.new) >= 1:
            a, b, t = self.new[0]
            if abs(a - self.last_commited_time) < 1:
                if self.commited_in_buffer:
                    cn, nn = len(self.commited_in_buffer), len(self.new)
                    for i in range(1, min(min(cn, nn), 5) + 1):
                        c = " ".join([self.commited_in_buffer[-j][2] for j in range(1, i + 1)][::-1])
                        tail = " ".join(self.new[j - 1][2] for j in range(1, i + 1))
                        if c == tail:
                            for _ in range(i):
                                self.new.pop(0)
                            break

    def flush(self):
        commit = []
        while self.new:
            na, nb, nt = self.new[0]
            if len(self.buffer) == 0:
                break
            if nt == self.buffer[0][2]:
                commit.append((na, nb, nt))
                self.last_commited_word = nt
                self.last_commited_time = nb
                self.buffer.pop(0)
                self.new.pop(0)
            else:
                break
        self.buffer = self.new
        self.new = []
        self.commited_in_buffer.extend(commit)
        return commit

    def pop_commited(self, time):
        while self.commited_in_buffer and self.commited_in_buffer[0][1] <= time:
            self.commited_in_buffer.pop(0)

    def complete(self):
        return self.buffer


class OnlineASRProcessor:
    SAMPLING_RATE = SAMPLING_RATE

    def __init__(self, asr, tokenizer=None, buffer_trimming=("segment", 15), logfile=sys.stderr):
        self.asr = asr
        self.tokenizer = tokenizer
        self.logfile = logfile
        self.init()
        self.buffer_trimming_way, self.buffer_trimming_sec = buffer_trimming

    def init(self, offset=None):
        self.audio_buffer = np.array([], dtype=np.float32)
        self.transcript_buffer = HypothesisBuffer(logfile=self.logfile)
        self.buffer_time_offset = 0
        if offset is not None:
            self.buffer_time_offset = offset
        self.transcript_buffer.last_commited_time = self.buffer_time_offset
        self.commited = []

    def insert_audio_chunk(self, audio):
        self.audio_buffer = np.append(self.audio_buffer, audio)

    def prompt(self):
        k = max(0, len(self.commited) - 1)
        while k > 0 and self.commited[k - 1][1] > self.buffer_time_offset:
            k -= 1
        p = [t for _, _, t in self.commited[:k]]
        prompt, n = [], 0
        while p and n < 200:
            x = p.pop(-1)
            n += len(x) + 1
            prompt.append(x)
        non_prompt = self.commited[k:]
        return self.asr.sep.join(prompt[::-1]), self.asr.sep.join(t for _, _, t in non_prompt)

    # process_iter split in two so a batcher can run many streams' transcribe calls as one launch
    def prepare_iter(self):
        prompt, _ = self.prompt()
        return self.audio_buffer, prompt

    def complete_iter(self, res):
        tsw = self.asr.ts_words(res)
        self.transcript_buffer.insert(tsw, self.buffer_time_offset)
        o = self.transcript_buffer.flush()
        self.commited.extend(o)
        if o and self.buffer_trimming_way == "sentence":
            if len(self.audio_buffer) / self.SAMPLING_RATE > self.buffer_trimming_sec:
                self.chunk_completed_sentence()
        s = self.buffer_trimming_sec if self.buffer_trimming_way == "segment" else 30
        if len(self.audio_buffer) / self.SAMPLING_RATE > s:
            self.chunk_completed_segment(res)
        return self.to_flush(o)

    def process_iter(self):
        audio, prompt = self.prepare_iter()
        res = self.asr.transcribe(audio, init_prompt=prompt)
        return self.complete_iter(res)

    def chunk_completed_sentence(self):
        if not self.commited or self.tokenizer is None:
            return
        sents = self.words_to_sentences(self.commited)
        if len(sents) < 2:
            return
        while len(sents) > 2:
            sents.pop(0)
        self.chunk_at(sents[-2][1])

    def chunk_completed_segment(self, res):
        if not self.commited:
            return
        ends = self.asr.segments_end_ts(res)
        t = self.commited[-1][1]
        if len(ends) > 1:
            e = ends[-2] + self.buffer_time_offset
            while len(ends) > 2 and e > t:
                ends.pop(-1)
                e = ends[-2] + self.buffer_time_offset
            if e <= t:
                self.chunk_at(e)

    def chunk_at(self, time):
        self.transcript_buffer.pop_commited(time)
        cut = time - self.buffer_time_offset
        self.audio_buffer = self.audio_buffer[int(cut * self.SAMPLING_RATE):]
        self.buffer_time_offset = time

    def words_to_sentences(self, words):
        cwords = list(words)
        t = " ".join(o[2] for o in cwords)
        s = self.tokenizer.split(t)
        out = []
        while s:
            beg = end = None
            sent = s.pop(0).strip()
            fsent = sent
            while cwords:
                b, e, w = cwords.pop(0)
                w = w.strip()
                if beg is None and sent.startswith(w):
                    beg = b
                elif end is None and sent == w:
                    end = e
                    out.append((beg, end, fsent))
                    break
                sent = sent[len(w):].strip()
        return out

    def finish(self):
        o = self.transcript_buffer.complete()
        f = self.to_flush(o)
        self.buffer_time_offset += len(self.audio_buffer) / SAMPLING_RATE
        return f

    def to_flush(self, sents, sep=None, offset=0):
        if sep is None:
            sep = self.asr.sep
        t = sep.join(s[2] for s in sents)
        if len(sents) == 0:
            return (None, None, t)
        return (offset + sents[0][0], offset + sents[-1][1], t)


# ------------------------------------------------------------------------------------------------
# VAD: silero_vad_iterator.VADIterator rules with a pluggable speech-probability model
# ------------------------------------------------------------------------------------------------
class EnergyVAD:
    """Stand-in for the Silero network (remote-only): speech probability from the 512-sample RMS."""

    def __init__(self, rms_mid=0.02, slope=200.0):
        self.rms_mid, self.slope = rms_mid, slope

    def reset_states(self):
        pass

    def __call__(self, x, sr=16000):
        rms = float(np.sqrt(np.mean(np.square(np.asarray(x, np.float64))))) if len(x) else 0.0
        return 1.0 / (1.0 + np.exp(-self.slope * (rms - self.rms_mid)))


class ScriptedVAD:
    """Deterministic probability track (tests / config 2 bench): probs[i] for the i-th 512-sample window."""

    def __init__(self, probs):
        self.probs = list(probs)
        self.i = 0

    def reset_states(self):
        self.i = 0

    def __call__(self, x, sr=16000):
        p = self.probs[self.i] if self.i < len(self.probs) else 0.0
        self.i += 1
        return p


class VADIterator:
    def __init__(self, model, threshold=0.5, sampling_rate=16000, min_silence_duration_ms=500, speech_pad_ms=100):
        self.model = model
        self.threshold = threshold
        self.sampling_rate = sampling_rate
        self.min_silence_samples = sampling_rate * min_silence_duration_ms / 1000
        self.speech_pad_samples = sampling_rate * speech_pad_ms / 1000
        self.reset_states()

    def reset_states(self):
        self.model.reset_states()
        self.triggered = False
        self.temp_end = 0
        self.current_sample = 0

    def __call__(self, x, return_seconds=False):
        n = len(x)
        self.current_sample += n
        p = self.model(x, self.sampling_rate)
        if p >= self.threshold and self.temp_end:
            self.temp_end = 0
        if p >= self.threshold and not self.triggered:
            self.triggered = True
            start = self.current_sample - self.speech_pad_samples - n
            return {"start": int(start) if not return_seconds else round(start / self.sampling_rate, 1)}
        if p < self.threshold - 0.15 and self.triggered:
            if not self.temp_end:
                self.temp_end = self.current_sample
            if self.current_sample - self.temp_end < self.min_silence_samples:
                return None
            end = self.temp_end + self.speech_pad_samples - n
            self.temp_end = 0
            self.triggered = False
            return {"end": int(end) if not return_seconds else round(end / self.sampling_rate, 1)}
        return None


class FixedVADIterator(VADIterator):
    """silero_vad_iterator.FixedVADIterator: arbitrary chunk lengths, 512-sample windows, merged events."""

    def reset_states(self):
        super().reset_states()
        self.buffer = np.array([], dtype=np.float32)

    def __call__(self, x, return_seconds=False):
        self.buffer = np.append(self.buffer, x)
        ret = None
        while len(self.buffer) >= 512:
            r = super().__call__(self.buffer[:512], return_seconds=return_seconds)
            self.buffer = self.buffer[512:]
            if ret is None:
                ret = r
            elif r is not None:
                if "end" in r:
                    ret["end"] = r["end"]
                if "start" in r and "end" in ret:
                    del ret["end"]
        return ret if ret != {} else None


class DynamicVADIterator:
    """Reference asr_components.py:12-78: FixedVADIterator with adjustable min_silence_samples."""

    def __init__(self, model, initial_silence_ms=500, min_silence_ms=200, max_silence_ms=1000, threshold=0.5):
        self.min_silence_ms = min_silence_ms
        self.max_silence_ms = max_silence_ms
        self.current_silence_ms = initial_silence_ms
        self.model = model
        self.threshold = threshold
        self.vad = VADIterator(model, threshold=threshold, min_silence_duration_ms=initial_silence_ms)
        self.buffer = np.array([], dtype=np.float32)

    def set_silence_duration(self, silence_ms):
        silence_ms = max(self.min_silence_ms, min(self.max_silence_ms, silence_ms))
        if abs(silence_ms - self.current_silence_ms) > 50:
            self.current_silence_ms = silence_ms
            self.vad.min_silence_samples = self.vad.sampling_rate * silence_ms / 1000
            return True
        return False

    def reset_states(self):
        self.vad.reset_states()
        self.buffer = np.array([], dtype=np.float32)

    def __call__(self, x, return_seconds=False):
        self.buffer = np.append(self.buffer, x)
        ret = None
        while len(self.buffer) >= 512:
            r = self.vad(self.buffer[:512], return_seconds=return_seconds)
            self.buffer = self.buffer[512:]
            if ret is None:
                ret = r
            elif r is not None:
                if "end" in r:
                    ret["end"] = r["end"]
                if "start" in r and "end" in ret:
                    del ret["end"]
        return ret if ret != {} else None


class VACOnlineASRProcessor(OnlineASRProcessor):
    """whisper_online.VACOnlineASRProcessor (reference restatement: asr_components.py:81-179)."""

    def __init__(self, online_chunk_size, asr, tokenizer=None, buffer_trimming=("segment", 15), logfile=sys.stderr,
                 vad=None, online=None):
        self.online_chunk_size = online_chunk_size
        self.online = online or OnlineASRProcessor(asr, tokenizer=tokenizer, logfile=logfile,
                                                   buffer_trimming=buffer_trimming)
        self.vac = vad or FixedVADIterator(EnergyVAD())
        self.logfile = logfile
        self.init()

    def init(self):
        self.online.init()
        self.vac.reset_states()
        self.current_online_chunk_buffer_size = 0
        self.is_currently_final = False
        self.status = None
        self.audio_buffer = np.array([], dtype=np.float32)
        self.buffer_offset = 0

    def clear_buffer(self):
        self.buffer_offset += len(self.audio_buffer)
        self.audio_buffer = np.array([], dtype=np.float32)

    def insert_audio_chunk(self, audio):
        res = self.vac(audio)
        self.audio_buffer = np.append(self.audio_buffer, audio)
        if res is not None:
            frame = list(res.values())[0] - self.buffer_offset
            if "start" in res and "end" not in res:
                self.status = "voice"
                send = self.audio_buffer[frame:]
                self.online.init(offset=(frame + self.buffer_offset) / self.SAMPLING_RATE)
                self.online.insert_audio_chunk(send)
                self.current_online_chunk_buffer_size += len(send)
                self.clear_buffer()
            elif "end" in res and "start" not in res:
                self.status = "nonvoice"
                send = self.audio_buffer[:frame]
                self.online.insert_audio_chunk(send)
                self.current_online_chunk_buffer_size += len(send)
                self.is_currently_final = True
                self.clear_buffer()
            else:
                beg = res["start"] - self.buffer_offset
                end = res["end"] - self.buffer_offset
                self.status = "nonvoice"
                send = self.audio_buffer[beg:end]
                self.online.init(offset=(beg + self.buffer_offset) / self.SAMPLING_RATE)
                self.online.insert_audio_chunk(send)
                self.current_online_chunk_buffer_size += len(send)
                self.is_currently_final = True
                self.clear_buffer()
        else:
            if self.status == "voice":
                self.online.insert_audio_chunk(self.audio_buffer)
                self.current_online_chunk_buffer_size += len(self.audio_buffer)
                self.clear_buffer()
            else:
                self.buffer_offset += max(0, len(self.audio_buffer) - self.SAMPLING_RATE)
                self.audio_buffer = self.audio_buffer[-self.SAMPLING_RATE:]

    def wants_iter(self):
        """True when process_iter() would run the ASR (used by the StreamBatcher)."""
        return (not self.is_currently_final) and \
            self.current_online_chunk_buffer_size > self.SAMPLING_RATE * self.online_chunk_size

    def process_iter(self):
        if self.is_currently_final:
            return self.finish()
        if self.current_online_chunk_buffer_size > self.SAMPLING_RATE * self.online_chunk_size:
            self.current_online_chunk_buffer_size = 0
            return self.online.process_iter()
        return (None, None, "")

    def finish(self):
        ret = self.online.finish()
        self.current_online_chunk_buffer_size = 0
        self.is_currently_final = False
        return ret


class DynamicVACOnlineASRProcessor(VACOnlineASRProcessor):
    """Reference asr_components.py:81-179 (DynamicVADIterator gate)."""

    def __init__(self, online_chunk_size, asr, tokenizer=None, logfile=sys.stderr, buffer_trimming=("segment", 15),
                 initial_silence_ms=500, min_silence_ms=200, max_silence_ms=1000, vad_threshold=0.5, vad_model=None,
                 online=None):
        if isinstance(vad_model, str):  # "silero" (synthetic weights) or a Silero v5 .safetensors path
            from .vad import silero_model
            vad_model = silero_model(vad_model)
        vad = DynamicVADIterator(vad_model or EnergyVAD(), initial_silence_ms, min_silence_ms, max_silence_ms,
                                 vad_threshold)
        super().__init__(online_chunk_size, asr, tokenizer=tokenizer, buffer_trimming=buffer_trimming,
                         logfile=logfile, vad=vad, online=online)

    def set_silence_duration(self, silence_ms):
        return self.vac.set_silence_duration(silence_ms)


# ------------------------------------------------------------------------------------------------
# reference enhancements (enhanced_asr_processor.py)
# ------------------------------------------------------------------------------------------------
class EnhancedHypothesisBuffer(HypothesisBuffer):
    """LocalAgreement-n (enhanced_asr_processor.py:32-156)."""

    def __init__(self, agreement_n=2, logfile=sys.stderr):
        super().__init__(logfile=logfile)
        self.agreement_n = agreement_n
        self.history = []
        self.max_history = agreement_n

    def insert(self, new, offset):
        super().insert(new, offset)
        state = self.buffer + self.new
        if len(self.history) >= self.max_history:
            self.history.pop(0)
        self.history.append(state.copy())

    def flush(self):
        if self.agreement_n == 2:
            return super().flush()
        if len(self.history) < self.agreement_n:
            self.buffer = self.buffer + self.new
            self.new = []
            return []
        recent = self.history[-self.agreement_n:]
        all_words = [[w for _, _, w in h] for h in recent]
        min_len = min(len(w) for w in all_words)
        common = 0
        for i in range(min_len):
            first = all_words[0][i]
            if all(w[i] == first for w in all_words):
                common += 1
            else:
                break
        commit = []
        if common > 0:
            last = recent[-1]
            for i in range(common):
                if i < len(last):
                    commit.append(last[i])
                    self.last_commited_word = last[i][2]
                    self.last_commited_time = last[i][1]
        if commit:
            for h in recent:
                for _ in range(common):
                    if h:
                        h.pop(0)
            self.commited_in_buffer.extend(commit)
        self.buffer = recent[-1].copy() if recent else []
        self.new = []
        return commit


class DynamicBufferManager:
    """enhanced_asr_processor.py:159-236 (trimming threshold 5-30 s driven by the recorded 'delay')."""

    def __init__(self, initial_trimming_sec=15, min_trimming_sec=5, max_trimming_sec=30):
        self.current_trimming_sec = initial_trimming_sec
        self.min_trimming_sec = min_trimming_sec
        self.max_trimming_sec = max_trimming_sec
        self.recent_delays = []
        self.recent_memory_usage = []
        self.max_delay_samples = 10
        self.max_memory_samples = 10

    def record_delay(self, delay):
        self.recent_delays.append(delay)
        if len(self.recent_delays) > self.max_delay_samples:
            self.recent_delays.pop(0)

    def record_memory_usage(self, usage_percent):
        self.recent_memory_usage.append(usage_percent)
        if len(self.recent_memory_usage) > self.max_memory_samples:
            self.recent_memory_usage.pop(0)

    def adjust_trimming_sec(self):
        if not self.recent_delays:
            return self.current_trimming_sec
        avg_delay = sum(self.recent_delays) / len(self.recent_delays)
        avg_mem = sum(self.recent_memory_usage) / len(self.recent_memory_usage) if self.recent_memory_usage else 50
        new = self.current_trimming_sec
        if avg_delay > 3.0 or avg_mem > 80.0:
            new = max(self.min_trimming_sec, self.current_trimming_sec - 2.0)
        elif avg_delay < 1.5 and avg_mem < 56.0:
            new = min(self.max_trimming_sec, self.current_trimming_sec + 2.0)
        if abs(new - self.current_trimming_sec) > 0.5:
            self.current_trimming_sec = new
            return True
        return False

    def get_trimming_sec(self):
        return self.current_trimming_sec


class EnhancedOnlineASRProcessor(OnlineASRProcessor):
    """enhanced_asr_processor.py:239-398: LocalAgreement-n, 300-char prompt, dynamic trimming, reset on error."""

    def __init__(self, asr, tokenizer=None, buffer_trimming=("segment", 15), logfile=sys.stderr, agreement_n=2,
                 enable_dynamic_buffer=True):
        self.asr = asr
        self.tokenizer = tokenizer
        self.logfile = logfile
        self.buffer_trimming_way, self.buffer_trimming_sec = buffer_trimming
        self.agreement_n = agreement_n
        self.enable_dynamic_buffer = enable_dynamic_buffer
        self.buffer_manager = DynamicBufferManager(self.buffer_trimming_sec, 5, 30) if enable_dynamic_buffer else None
        self.init()

    def init(self, offset=None):
        self.audio_buffer = np.array([], dtype=np.float32)
        self.transcript_buffer = EnhancedHypothesisBuffer(agreement_n=self.agreement_n, logfile=self.logfile)
        self.buffer_time_offset = 0 if offset is None else offset
        self.transcript_buffer.last_commited_time = self.buffer_time_offset
        self.commited = []

    def prompt(self):
        prompt_parts, plen = [], 0
        for item in reversed(self.commited):
            word = item[2]
            wl = len(word) + 1
            if plen + wl > 300:
                break
            prompt_parts.append(word)
            plen += wl
        prompt = self.asr.sep.join(reversed(prompt_parts))
        non_prompt_parts, nlen = [], 0
        pw = set(prompt_parts)
        for item in reversed(self.commited):
            word = item[2]
            if word not in pw:
                wl = len(word) + 1
                if nlen + wl > 500:
                    break
                non_prompt_parts.append(word)
                nlen += wl
        return prompt, self.asr.sep.join(reversed(non_prompt_parts))

    def prepare_iter(self):
        if self.enable_dynamic_buffer and self.buffer_manager:
            if self.buffer_manager.adjust_trimming_sec():
                self.buffer_trimming_sec = self.buffer_manager.get_trimming_sec()
        return super().prepare_iter()

    def complete_iter(self, res):
        result = super().complete_iter(res)
        if self.enable_dynamic_buffer and self.buffer_manager and result[0] is not None:
            # the reference records the buffer duration as the "delay" (enhanced_asr_processor.py:362-365)
            self.buffer_manager.record_delay(len(self.audio_buffer) / self.SAMPLING_RATE)
        return result

    def process_iter(self):
        try:
            audio, prompt = self.prepare_iter()
            res = self.asr.transcribe(audio, init_prompt=prompt)
            return self.complete_iter(res)
        except Exception as e:  # enhanced_asr_processor.py:369-381
            print(f"process_iter error: {e}", file=self.logfile)
            try:
                self.init(offset=self.buffer_time_offset)
            except Exception:
                pass
            return (None, None, "")

    def set_agreement_n(self, n):
        self.agreement_n = max(2, n)
        self.transcript_buffer = EnhancedHypothesisBuffer(agreement_n=self.agreement_n, logfile=self.logfile)
        self.transcript_buffer.last_commited_time = self.buffer_time_offset


class EnhancedVACOnlineASRProcessor(VACOnlineASRProcessor):
    """enhanced_asr_processor.py:401-502."""

    def __init__(self, online_chunk_size, asr, tokenizer=None, logfile=sys.stderr, buffer_trimming=("segment", 15),
                 agreement_n=2, enable_dynamic_buffer=True, initial_silence_ms=500, min_silence_ms=200,
                 max_silence_ms=1000, vad_threshold=0.5, vad_model=None):
        online = EnhancedOnlineASRProcessor(asr=asr, tokenizer=tokenizer, logfile=logfile,
                                            buffer_trimming=buffer_trimming, agreement_n=agreement_n,
                                            enable_dynamic_buffer=enable_dynamic_buffer)
        if isinstance(vad_model, str):  # "silero" (synthetic weights) or a Silero v5 .safetensors path
            from .vad import silero_model
            vad_model = silero_model(vad_model)
        vad = DynamicVADIterator(vad_model or EnergyVAD(), initial_silence_ms, min_silence_ms, max_silence_ms,
                                 vad_threshold)
        super().__init__(online_chunk_size, asr, tokenizer=tokenizer, buffer_trimming=buffer_trimming,
                         logfile=logfile, vad=vad, online=online)

    def set_silence_duration(self, silence_ms):
        return self.vac.set_silence_duration(silence_ms)

    def set_agreement_n(self, n):
        self.online.set_agreement_n(n)


# ------------------------------------------------------------------------------------------------
# multi-stream batching (data parallel over independent streams, one GPU)
# ------------------------------------------------------------------------------------------------
# decoding options the batched multi-stream path carries; anything else in a stream's options raises
_BATCH_KWARGS = ("task", "beam_size", "temperature", "best_of")


def batch_transcribe_kwargs(asr):
    """The decoding options one batched call uses, merged as CustomFasterWhisperASR.transcribe merges them
    (asr_components.py:270-275): the ASR's transcribe_kargs, overridden by adaptive_params.get_transcribe_kwargs()
    (speech_rate_audio_processor.py:234-237: beam size / temperature per call) when the ASR has adaptive params.
    Options the batched path does not implement raise instead of being dropped."""
    kw = dict(getattr(asr, "transcribe_kargs", None) or {})
    ap = getattr(asr, "adaptive_params", None)
    if ap:
        kw.update(ap.get_transcribe_kwargs())
    extra = sorted(k for k in kw if k not in _BATCH_KWARGS)
    if extra:
        raise NotImplementedError(f"StreamBatcher: transcribe options {extra} are not implemented on the batched "
                                  f"multi-stream path (supported: {list(_BATCH_KWARGS)})")
    return kw


class StreamBatcher:
    """Runs the due process_iter() of many VAC streams as one batched transcribe on one MI355X.

    `model` is a wmx.transcribe.WhisperModel whose max_batch >= number of streams; windows must be <= 30 s
    (the streaming buffers are trimmed at 5-30 s).  Each stream keeps its own buffers / LocalAgreement state;
    only the ASR call is shared."""

    def __init__(self, model, asr_view):
        self.model = model
        self.asr = asr_view  # provides ts_words / segments_end_ts / sep for the per-stream completion

    def step(self, streams):
        due, outs = [], [None] * len(streams)
        for i, s in enumerate(streams):
            if s.is_currently_final:
                outs[i] = s.finish()
            elif s.wants_iter():
                s.current_online_chunk_buffer_size = 0
                due.append(i)
            else:
                outs[i] = (None, None, "")
        if due:
            reqs = [streams[i].online.prepare_iter() for i in due]
            kw = batch_transcribe_kwargs(self.asr)
            results = self.model.transcribe_batch([a for a, _ in reqs], [p for _, p in reqs],
                                                  language=getattr(self.asr, "original_language", None),
                                                  task=kw.get("task", "transcribe"), beam_size=kw.get("beam_size"),
                                                  temperature=kw.get("temperature", 0.0) or 0.0,
                                                  best_of=kw.get("best_of", 5))
            for i, res in zip(due, results):
                on = streams[i].online
                try:
                    if isinstance(res, Exception):
                        raise res
                    outs[i] = on.complete_iter(res)
                except Exception as e:  # per stream, EnhancedOnlineASRProcessor.process_iter (:369-381)
                    print(f"process_iter error: {e}", file=getattr(on, "logfile", sys.stderr))
                    try:
                        on.init(offset=on.buffer_time_offset)
                    except Exception:
                        pass
                    outs[i] = (None, None, "")
        return outs
