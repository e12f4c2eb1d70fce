"""Drop-in ASR backend for the reference's plugin surface.

Mirrors `CustomFasterWhisperASR` (reference asr_components.py:182-311) — same constructor keywords, same
methods (`transcribe`, `ts_words`, `segments_end_ts`, `set_translate_task`, `use_vad`), same attribute `sep`
(faster-whisper's whisper_online.FasterWhisperASR uses ""), same error flow (exceptions propagate to
OnlineASRProcessor.process_iter) — but the engine below is libwmx.so on MI355X instead of
faster-whisper/CTranslate2.

    from wmx.asr import MI355XWhisperASR
    asr = MI355XWhisperASR(lan="auto", modelsize="large-v3", device="cuda", compute_type="float16")
    online = EnhancedOnlineASRProcessor(asr, ...)        # unchanged caller
"""
from __future__ import annotations

import sys

from .transcribe import WhisperModel


class MI355XWhisperASR:
    sep = ""  # whisper_online.FasterWhisperASR.sep (faster-whisper words carry their own leading space)

    def __init__(self, lan, modelsize=None, cache_dir=None, model_dir=None, device="cuda", compute_type="float16",
                 device_index=0, num_workers=1, cpu_threads=None, logfile=sys.stderr, adaptive_params=None,
                 transcribe_kwargs=None, seed=1, max_new_tokens=None):
        # asr_components.py:195-230
        self.device = device
        self.compute_type = compute_type
        self.device_index = device_index
        self.num_workers = num_workers
        self.cpu_threads = cpu_threads
        self.logfile = logfile
        self.transcribe_kargs = transcribe_kwargs if transcribe_kwargs else {}
        self.adaptive_params = adaptive_params
        self.original_language = None if lan == "auto" else lan
        self._seed = seed
        self._max_new_tokens = max_new_tokens
        self.model = self.load_model(modelsize, cache_dir, model_dir)

    def load_model(self, modelsize=None, cache_dir=None, model_dir=None):
        # asr_components.py:232-265 (GPU branch; the CPU/int8 fallback of the app is not a MI355X path)
        if model_dir is not None:
            name = model_dir
        elif modelsize is not None:
            name = modelsize
        else:
            raise ValueError("modelsize or model_dir parameter must be set")
        if self.device == "cpu":
            # the app's CPU/int8 fallback (asr_components.py:256-258) has no MI355X engine: fail loudly
            raise ValueError("MI355XWhisperASR runs on the GPU only (device='cuda'); there is no CPU/int8 path")
        # the faster-whisper WhisperModel kwargs of asr_components.py:244-254, then the engine's own keys
        model_kwargs = {"device": self.device, "compute_type": self.compute_type, "download_root": cache_dir,
                        "num_workers": self.num_workers, "device_index": self.device_index}
        return WhisperModel(name, **model_kwargs, seed=self._seed,
                            beam_size=self.transcribe_kargs.get("beam_size", 5), max_new_tokens=self._max_new_tokens)

    def transcribe(self, audio, init_prompt=""):
        # asr_components.py:267-289: adaptive kwargs merged over transcribe_kargs; word_timestamps and
        # condition_on_previous_text forced on; beam_size / temperature default 5 / 0.0
        if self.adaptive_params:
            kw = {**self.transcribe_kargs, **self.adaptive_params.get_transcribe_kwargs()}
        else:
            kw = self.transcribe_kargs
        segments, info = self.model.transcribe(
            audio, language=self.original_language, initial_prompt=init_prompt,
            beam_size=kw.get("beam_size", 5), temperature=kw.get("temperature", 0.0), word_timestamps=True,
            condition_on_previous_text=True, **{k: v for k, v in kw.items() if k not in ("beam_size", "temperature")})
        return list(segments)

    def ts_words(self, segments):
        # asr_components.py:291-297 (the override does NOT filter no-speech segments)
        o = []
        for s in segments:
            for word in s.words:
                o.append((word.start, word.end, word.word))
        return o

    def segments_end_ts(self, segments):
        return [s.end for s in segments]

    def set_translate_task(self):
        self.transcribe_kargs["task"] = "translate"

    def use_vad(self):
        self.transcribe_kargs["vad_filter"] = True


def create_custom_faster_whisper_asr(FasterWhisperASR=None):
    """Same factory shape as asr_components.py:182: the parent class argument is accepted and ignored."""
    return MI355XWhisperASR
