"""Replays the decode step's reduce_ln launch alone (8 windows x beam 5 of large-v3 = 40 rows in one context, the
split count of the d x d projection) for PMC passes:
rocprofv3 --kernel-include-regex reduce_ln --pmc <counters> -- python tools/redln_pmc.py [--batch B]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "realtime-whisper-asr_amd"))
import torch  # noqa: E402

torch.cuda.init()
from wmx import engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4)
args = ap.parse_args()
m = engine.Model("large-v3", 0, "bfloat16")
ctx = engine.Context(m, max_batch=args.batch, beam_size=5, max_new_tokens=8)
ms, by, _ = ctx.bench_kernel("reduce_ln", args.batch, iters=20)
print(f"reduce_ln {1000 * ms:.2f} us/launch, {by / ms / 1e6:.1f} GB/s", flush=True)
