"""One large-v3 encoder pass over B windows (bf16 or float8) for rocprofv3 --kernel-trace breakdowns.
Usage: python tools/encprof_b.py <bfloat16|float8> <B>"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "realtime-whisper-asr_amd"))
import torch  # noqa: E402

torch.cuda.init()
from wmx.engine import Context, Model  # noqa: E402

ct = sys.argv[1] if len(sys.argv) > 1 else "bfloat16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
m = Model("large-v3", 0, ct)
ctx = Context(m, max_batch=B, beam_size=1, max_new_tokens=8)
ms, _, fl = ctx.bench_kernel("encoder", B, iters=3)
print(f"{ct} B={B}: encoder {ms:.2f} ms {fl / ms / 1e9:.1f} TFLOP/s")
