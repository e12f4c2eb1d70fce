"""Replays the encoder attention kernel alone (8 windows of large-v3, synthetic weights) for PMC passes:
rocprofv3 --pmc <counters> -- python tools/attn_pmc.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "realtime-whisper-asr_amd"))
import torch  # noqa: E402

torch.cuda.init()
from wmx import engine  # noqa: E402

m = engine.Model("large-v3", 0, "bfloat16")
m.init_synthetic(1)
ctx = engine.Context(m, max_batch=8, beam_size=1, max_new_tokens=8)
ms, _, fl = ctx.bench_kernel("enc_attn", 8, iters=5)
print(f"enc_attn {1000 * ms:.1f} us {fl / ms / 1e9:.1f} TF/s", flush=True)
