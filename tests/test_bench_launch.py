"""bench.py --gpus N outside torch.distributed.run: the parent spawns N rank processes (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* in their environment, before any torch / HIP call in the parent), the ranks rendezvous,
broadcast the arena from rank 0, time barrier-bracketed steps, reduce the max over ranks through wmx.dist, and the
parent relays rank 0's single JSON line.  Driven here with --dry-run (gloo, host stand-in step, no GPU): the same
launcher and wmx.dist calls the GPU run makes, with the RCCL backend swapped for gloo."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_spawned_ranks_report_one_line(n):
    out = _run("--gpus", str(n), "--dry-run", "--steps", "2", "--warmup", "1")
    assert out["n_gpus"] == n and out["ranks_reporting"] == n and out["arena_broadcast_ok"] is True
    assert out["scaling"] == "weak" and out["value"] > 0


def test_single_gpu_path_unchanged():
    out = _run("--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "0")
    assert out["n_gpus"] == 1 and out["ranks_reporting"] == 1
