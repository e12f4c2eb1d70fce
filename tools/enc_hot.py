"""Encoder pass time (8 windows, HIP events) cool, right after decode-heavy transcribes, and after an idle pause:
separates the chip's clock state from kernel changes.  Run on the GPU box."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "realtime-whisper-asr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from wmx import engine, synth  # noqa: E402

m = engine.Model("large-v3", 0, sys.argv[1] if len(sys.argv) > 1 else "bfloat16")
m.init_synthetic(1)
ctx = engine.Context(m, max_batch=8, beam_size=5, max_new_tokens=224, language=None, word_timestamps=True,
                     alignment_heads=engine.ALIGNMENT_HEADS.get("large-v3"))
audio = np.stack([synth.speech_like(i, 480000) for i in range(8)])
pcm = torch.from_numpy(audio).cuda()
lens = np.full(8, 480000, np.int64)


def enc(tag):
    ms, _, fl = ctx.bench_kernel("encoder", 8, iters=3)
    print(f"{tag:28s} encoder {ms:6.2f} ms  {fl / ms / 1e9:7.1f} TF/s  {fl / ms / 1e9 / 2500:.3f}", flush=True)


enc("cool")
enc("cool again")
for i in range(3):
    t = time.time()
    ctx.transcribe_device(pcm.data_ptr(), 480000, lens)
    torch.cuda.synchronize()
    print(f"transcribe {i}: {time.time() - t:.2f} s", flush=True)
enc("after decode")
enc("after decode, again")
time.sleep(5)
enc("after 5 s idle")
