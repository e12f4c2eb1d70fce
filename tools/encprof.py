"""One large-v3 encoder pass over 8 windows (bf16 or float8), for rocprofv3 --kernel-trace breakdowns."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "realtime-whisper-asr_amd"))
import torch  # noqa: E402

torch.cuda.init()
from wmx.engine import Context, Model  # noqa: E402

ct = sys.argv[1] if len(sys.argv) > 1 else "bfloat16"
m = Model("large-v3", 0, ct)
m.init_synthetic(1)  # random weights: zero-filled operands run ~10 % faster (DVFS), not representative
ctx = Context(m, max_batch=8, beam_size=1, max_new_tokens=8)
ms, _, fl = ctx.bench_kernel("encoder", 8, iters=3)
print(f"{ct}: encoder {ms:.2f} ms {fl / ms / 1e9:.1f} TFLOP/s")
