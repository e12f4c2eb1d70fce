"""Localise a concurrency-dependent result difference: two contexts on one model, each stage run from two host
threads at once and compared bit for bit with the same stage run alone (log-mel, encoder, whole transcribe without
and with the lockstep barrier).  Usage: python tools/conc_probe.py [reps]"""
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
ctxs = [E.Context(m, max_batch=2, beam_size=5, max_new_tokens=24, language=None, word_timestamps=True,
                  use_graph=True) for _ in range(2)]
audios = [synth.speech_like(950 + i, 480000) for i in range(4)]
batches = [audios[:2], audios[2:]]


def both(fn):
    out, err = [None, None], []
    go = threading.Barrier(2)

    def work(i):
        try:
            go.wait()
            out[i] = fn(i)
        except Exception as e:
            err.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    return out


def key(res):
    return [(tuple(r.tokens), r.sum_logprob, r.no_speech_prob, r.language) for r in res]


mel_ref = [ctxs[g].logmel(batches[g]) for g in range(2)]
bad = sum(not all(np.array_equal(a, b) for a, b in zip(both(lambda g: ctxs[g].logmel(batches[g])), mel_ref))
          for _ in range(REPS))
print(f"logmel: {bad} / {REPS} concurrent reps differ", flush=True)
enc_ref = [ctxs[g].encode(mel_ref[g]) for g in range(2)]
bad = sum(not all(np.array_equal(a, b) for a, b in zip(both(lambda g: ctxs[g].encode(mel_ref[g])), enc_ref))
          for _ in range(REPS))
print(f"encode: {bad} / {REPS} concurrent reps differ", flush=True)
tr_ref = [key(ctxs[g].transcribe(batches[g])) for g in range(2)]
bad = sum(not all(key(a) == b for a, b in zip(both(lambda g: ctxs[g].transcribe(batches[g])), tr_ref))
          for _ in range(REPS))
print(f"transcribe (no lockstep): {bad} / {REPS} concurrent reps differ", flush=True)
for c in ctxs:
    c.set_lockstep(21, 2)
bad = 0
for _ in range(REPS):
    got = both(lambda g: ctxs[g].transcribe(batches[g]))
    diff = [g for g in range(2) if key(got[g]) != tr_ref[g]]
    bad += bool(diff)
    if diff:
        g = diff[0]
        print("   differ: group", g, [(a[1], b[1]) for a, b in zip(key(got[g]), tr_ref[g])], flush=True)
print(f"transcribe (lockstep): {bad} / {REPS} concurrent reps differ", flush=True)
for c in ctxs:
    c.set_lockstep(0, 0)
# alone again: does a single context reproduce its own reference call after call?
bad = sum(key(ctxs[0].transcribe(batches[0])) != tr_ref[0] for _ in range(REPS))
print(f"transcribe alone: {bad} / {REPS} reps differ", flush=True)

# with the search recorder on: the first decode step whose raw logits differ from the alone reference
for c in ctxs:
    c.record(24)
ref_lg = []
for g in range(2):
    ctxs[g].transcribe(batches[g])
    ref_lg.append(ctxs[g].recorded()[0].copy())
bad = 0
for rep in range(REPS):
    both(lambda g: ctxs[g].transcribe(batches[g]))
    for g in range(2):
        lg = ctxs[g].recorded()[0]
        if not np.array_equal(lg, ref_lg[g]):
            bad += 1
            steps = [i for i in range(lg.shape[0]) if not np.array_equal(lg[i], ref_lg[g][i])]
            i = steps[0]
            rows = [r for r in range(lg.shape[1]) if not np.array_equal(lg[i, r], ref_lg[g][i, r])]
            print(f"   rep {rep} group {g}: first differing step {i} of {lg.shape[0]} (steps {steps[:8]}), rows {rows}, "
                  f"max |diff| {float(np.max(np.abs(lg[i] - ref_lg[g][i]))):.3e}", flush=True)
print(f"recorded logits (no lockstep): {bad} differing group-calls in {REPS} reps", flush=True)
