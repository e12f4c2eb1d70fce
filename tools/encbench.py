import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "realtime-whisper-asr_amd"))
import torch
torch.cuda.init()
from wmx.engine import Model, Context
for ct in ("bfloat16", "float8"):
    m = Model("large-v3", 0, ct)
    m.init_synthetic(1)  # random weights: zero-filled operands run ~10 % faster (DVFS), not representative
    ctx = Context(m, max_batch=8, beam_size=1, max_new_tokens=8)
    for B in (4, 8):
        ms, by, fl = ctx.bench_kernel("encoder", B, iters=3)
        print(f"{ct} B={B}: encoder {ms:.2f} ms  {fl/ms/1e9:.1f} TFLOP/s", flush=True)
    del ctx
    m.close()
