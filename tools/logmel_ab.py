import os, sys, json
sys.path[:0] = [os.environ.get("GRAFT_REPO_ROOT", "."), os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "realtime-whisper-asr_amd")]
import torch; torch.cuda.init()
from wmx.engine import Context, Model
m = Model("large-v3", 0, "bfloat16"); m.init_synthetic(1)
ctx = Context(m, max_batch=8, beam_size=1, max_new_tokens=8, word_timestamps=False)
for B in (4, 8):
    ms, by, fl = ctx.bench_kernel("logmel", B, iters=50)
    print(json.dumps({"gemm": bool(os.environ.get("WMX_LOGMEL_GEMM")), "B": B, "us": round(ms * 1000, 1), "gbs": round(by / ms / 1e6, 1), "tflops": round(fl / ms / 1e9, 2)}))
