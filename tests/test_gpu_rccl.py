"""The RCCL weight-broadcast path of the multi-GPU bench (bench.py -> wmx.dist.share_weights), executed
on one GPU before any 8-GPU node runs it.

A child process (torch first, so that it and libwmx share one HIP runtime, as bench.py does) joins a world-size-1
torch.distributed group over `nccl` (RCCL), builds a source model from the PRNG and an uninitialised destination
model, copies the source arena into the destination's through the zero-copy arena views (a device copy standing in
for the xGMI transfer a second rank receives), runs the RCCL broadcast on the destination's arena exactly as
share_weights does, marks it loaded (which re-derives the row-major and MX-fp8 copies) and transcribes with both:
the tokens, scores and jump times must be identical.  bf16 and float8 (config 5: the MX-fp8 and 8-bit copies are
derived after the load).  The broadcast carries the arena's PARAMETER region only: its byte count is the parameters'
16-bit bytes plus the fp32 biases / LayerNorms and the encoder positions (<= 2 B x n_params x 1.02 + 1500 x d x 4),
whatever the dtype -- the derived row-major / MX-fp8 / 8-bit copies (+50 % or more) are rebuilt on the receiving rank.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
import torch
import numpy as np
sys.path[:0] = [os.path.join(os.environ["WMX_ROOT"], "realtime-whisper-asr_amd"), os.environ["WMX_ROOT"]]
torch.cuda.set_device(0)
torch.zeros(1, device="cuda:0")
from wmx import dist as D, engine as E, synth
dev = torch.device("cuda", 0)
D.init("nccl", dev)
out = {}
for ct in ("bfloat16", "float8"):
    dims = E.ModelDims(128, 51866, 1280, 20, 2, 1280, 20, 2)
    src = E.Model(dims, 0, ct).init_synthetic(21)
    dst = E.Model(dims, 0, ct)
    vs, vd = D.arena_tensor(src, dev), D.arena_tensor(dst, dev)
    assert vs.numel() == vd.numel() and vs.data_ptr() != vd.data_ptr()
    vd.copy_(vs)
    D.share_weights(dst, 0, dev)  # RCCL broadcast of the arena + mark loaded
    audios = [synth.speech_like(40 + i, 480000) for i in range(2)]
    res = []
    for m in (src, dst):
        ctx = E.Context(m, max_batch=2, beam_size=5, max_new_tokens=24, word_timestamps=True, language=None)
        res.append(ctx.transcribe(audios))
        ctx.close()
    same = all(a.tokens == b.tokens and a.sum_logprob == b.sum_logprob and
               np.array_equal(a.jump_times, b.jump_times) for a, b in zip(*res))
    out[ct] = {"same": bool(same), "tokens": [len(r.tokens) for r in res[1]], "arena_bytes": int(vd.numel()),
               "arena_equal": bool(torch.equal(vs, vd)), "n_params": int(src.n_params())}
    dst.close(); src.close()
D.destroy()
print("RESULT " + json.dumps(out))
"""


def test_rccl_arena_broadcast_world1():
    env = dict(os.environ, WMX_ROOT=ROOT, MASTER_ADDR="127.0.0.1", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    from wmx.dist import free_port
    env["MASTER_PORT"] = str(free_port())
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    out = json.loads(line[7:])
    print(out)
    for ct, v in out.items():
        assert v["same"] and v["arena_equal"], (ct, v)
        assert min(v["tokens"]) == 24, (ct, v)
        assert 2 * v["n_params"] <= v["arena_bytes"] <= 2.04 * v["n_params"] + 1500 * 1280 * 4, (ct, v)
    assert out["bfloat16"]["arena_bytes"] == out["float8"]["arena_bytes"], out
