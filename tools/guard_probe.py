"""Out-of-bounds write finder (WMX_GUARD=1): the concurrent workload of tools/conc_probe4.py (context A transcribes while context B encodes,
and each alone) with a guard gap after every arena buffer; reports the first buffer whose gap was overwritten."""
import ctypes as C
import os
import sys
import threading

os.environ["WMX_GUARD"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "realtime-whisper-asr_amd"), ROOT]

from oracle import whisper_np as O  # noqa: E402
from wmx import engine as E  # noqa: E402
from wmx import synth  # noqa: E402
from wmx._lib import check, lib  # noqa: E402

d = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 2)
sp = O.special_tokens(d.n_vocab)
m = E.Model(E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                        d.n_text_head, d.n_text_layer), 0, "bfloat16").init_synthetic(6)
audios = [synth.speech_like(950 + i, 480000) for i in range(4)]
batches = [audios[:2], audios[2:]]
A, Bc = [E.Context(m, max_batch=2, beam_size=5, max_new_tokens=24, use_graph=True, language=sp.lang0,
                   word_timestamps=True) for _ in range(2)]


def gc(tag):
    for name, ctx in (("A", A), ("B", Bc)):
        mb, cb = C.c_int(), C.c_int()
        check(lib.wmx_debug_guard_check(m._h, ctx._h, C.byref(mb), C.byref(cb)))
        print(f"{tag}: model buffer {mb.value}, context {name} buffer {cb.value}", flush=True)


gc("created")
A.logmel(batches[0])
gc("after A logmel")
mel = A.logmel(batches[0])
A.encode(mel, want_output=False)
gc("after A encode")
A.transcribe(batches[0])
gc("after A transcribe")
Bc.encode(mel, want_output=False)
gc("after B encode")
stop = threading.Event()
t = threading.Thread(target=lambda: [Bc.encode(mel, want_output=False) for _ in iter(stop.is_set, True)])
t.start()
for _ in range(5):
    A.transcribe(batches[0])
stop.set()
t.join()
gc("after A transcribe | B encode")
