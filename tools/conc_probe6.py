"""Which of context B's encoder kernels, replayed in a loop (wmx_ctx_bench_kernel), perturbs context A's log-mel
(tools/conc_probe4.py).  Usage: python tools/conc_probe6.py [reps]"""
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
m = E.Model(E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                        d.n_text_head, d.n_text_layer), 0, "bfloat16").init_synthetic(6)
audios = [synth.speech_like(950 + i, 480000) for i in range(4)]
A, Bc = [E.Context(m, max_batch=2, beam_size=5, max_new_tokens=24, use_graph=False, language=50259,
                   word_timestamps=False) for _ in range(2)]
mel_ref = A.logmel(audios[:2])
Bc.transcribe(audios[2:])  # (the replays use the geometry and data of the last transcribe)


def against(fb, tag):
    bad = 0
    for _ in range(REPS):
        stop = threading.Event()
        t = threading.Thread(target=lambda: [fb() for _ in iter(stop.is_set, True)])
        t.start()
        try:
            got = A.logmel(audios[:2])
        finally:
            stop.set()
            t.join()
        bad += not np.array_equal(got, mel_ref)
    print(f"A log-mel | B {tag}: {bad} / {REPS} differ", flush=True)


for k in ("encoder", "enc_fc1", "enc_attn", "logmel"):
    against(lambda: Bc.bench_kernel(k, 2, iters=5), k)
