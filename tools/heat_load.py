"""Keeps the GPU busy with back-to-back 8-window bf16 encoder passes for the given number of seconds (a heavy,
sustained load before a bench run: tests whether the decode's slow mode follows the chip's thermal / clock state).
Usage: python tools/heat_load.py <seconds>"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "realtime-whisper-asr_amd"))
import torch  # noqa: E402

torch.cuda.init()
from wmx import engine  # noqa: E402

m = engine.Model("large-v3", 0, "bfloat16").init_synthetic(1)
ctx = engine.Context(m, max_batch=8, beam_size=1, max_new_tokens=8)
t0, n = time.time(), 0
while time.time() - t0 < float(sys.argv[1]):
    ms, _, _ = ctx.bench_kernel("encoder", 8, iters=10)
    n += 10
    if n % 100 == 0:
        print(f"{time.time() - t0:6.1f} s: {n} passes, last {ms:.2f} ms", flush=True)
print(f"heat load: {n} encoder passes in {time.time() - t0:.1f} s, last {ms:.2f} ms", flush=True)
