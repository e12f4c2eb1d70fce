"""CPU oracle for the streaming-Whisper hot path — TEST INFRASTRUCTURE ONLY.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker (or the timed CPU baseline), never as the thing measured.

What it restates (the reference's arithmetic lives in un-vendored third-party
packages):

* faster-whisper 1.2.1 ``FeatureExtractor`` (log-mel, ``padding=160``) and
  ``pad_or_trim`` — called by the reference at ``asr_components.py:279``.
* The Whisper encoder / decoder forward (openai-whisper / CTranslate2 4.6.1
  semantics: pre-LN, exact-erf GELU, k_proj without bias, tied output embedding).
* openai-whisper decoding rules that CTranslate2 re-implements: SuppressBlank,
  SuppressTokens, ApplyTimestampRules (+ max_initial_timestamp), greedy and
  beam search with patience, language detection, no_speech_prob.
* openai-whisper ``find_alignment`` (alignment heads -> softmax -> std/mean
  normalise -> median filter 7 -> DTW) used for ``word_timestamps=True``
  (``asr_components.py:285``).

* (``dsp_np``) the pre-ASR DSP of the microphone loop: scipy.signal.filtfilt of
  the order-4 Butterworth band-pass (``vocal_separation.py:335-358``) and the
  audio-dedup feature vector (``audio_deduplicator.py:60-160``), pinned against
  the reference modules' own outputs (``tests/golden/make_dsp_golden.py`` imports
  them; they need only numpy / scipy).

Pinning: see ``tests/golden/make_golden.py`` — the log-mel, encoder, decoder
logits, DTW and median filter are checked against transformers 5.15.0's
independent Whisper implementation on seeded inputs / build-owned random
weights.  The reference repo itself ships no fixtures, so
decode-rule parity with CTranslate2 is "parity unpinned" beyond those.
"""
