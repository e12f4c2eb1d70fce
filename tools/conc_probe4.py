"""A's log-mel and encoder outputs while context B encodes in a loop (two contexts on one model, see tools/conc_probe.py)."""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "realtime-whisper-asr_amd"), ROOT]

from oracle import whisper_np as O  # noqa: E402
from wmx import engine as E  # noqa: E402
from wmx import synth  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
d = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 2)
sp = O.special_tokens(d.n_vocab)
m = E.Model(E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                        d.n_text_head, d.n_text_layer), 0, "bfloat16").init_synthetic(6)
audios = [synth.speech_like(950 + i, 480000) for i in range(4)]
A, Bc = [E.Context(m, max_batch=2, beam_size=5, max_new_tokens=24, use_graph=True, language=sp.lang0,
                   word_timestamps=False) for _ in range(2)]
mel_ref = A.logmel(audios[:2])
mel_b = Bc.logmel(audios[2:])
enc_ref = A.encode(mel_ref)
Bc.encode(mel_b, want_output=False)


def against(fa, check, tag):
    bad, worst = 0, 0.0
    for _ in range(REPS):
        stop = threading.Event()
        t = threading.Thread(target=lambda: [Bc.encode(mel_b, want_output=False) for _ in iter(stop.is_set, True)])
        t.start()
        try:
            got = fa()
        finally:
            stop.set()
            t.join()
        ok, w = check(got)
        bad += not ok
        worst = max(worst, w)
    print(f"{tag}: {bad} / {REPS} differ (max |diff| {worst:.3e})", flush=True)


def cmp(ref):
    return lambda g: (np.array_equal(g, ref), float(np.max(np.abs(g - ref))))


against(lambda: A.logmel(audios[:2]), cmp(mel_ref), "A log-mel | B encode")
against(lambda: A.encode(mel_ref), cmp(enc_ref), "A encode | B encode")
against(lambda: A.encode(A.logmel(audios[:2])), cmp(enc_ref), "A log-mel + encode | B encode")
