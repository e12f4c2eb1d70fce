"""Encoder pass (8 windows, random weights, HIP events) of the library at WMX_LIB, repeated: for interleaved A/B
runs of encoder kernels.  Usage: WMX_LIB=... python tools/enc_ab.py [bfloat16|float8]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "realtime-whisper-asr_amd"))
import torch  # noqa: E402

torch.cuda.init()
from wmx import engine  # noqa: E402

ct = sys.argv[1] if len(sys.argv) > 1 else "bfloat16"
m = engine.Model("large-v3", 0, ct)
m.init_synthetic(1)
ctx = engine.Context(m, max_batch=8, beam_size=1, max_new_tokens=8)
best = None
for _ in range(3):
    ms, _, fl = ctx.bench_kernel("encoder", 8, iters=3)
    best = ms if best is None else min(best, ms)
at, _, afl = ctx.bench_kernel("enc_attn", 8, iters=20)
print(f"{os.path.basename(os.environ.get('WMX_LIB', 'libwmx.so'))} {ct}: encoder {best:.2f} ms "
      f"{fl / best / 1e9:.1f} TF/s {fl / best / 1e9 / 2500:.4f}; enc_attn {1000 * at:.1f} us "
      f"{afl / at / 1e9:.1f} TF/s", flush=True)
