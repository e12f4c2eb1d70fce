"""Multi-GPU plumbing: one process per GPU, independent streams sharded by rank, the weight arena
broadcast once from rank 0 (RCCL over xGMI on MI355X, gloo in CPU tests), max-over-ranks timing.
There is no per-step collective: streams never exchange data.

`launch_ranks` is the single-node launcher bench.py uses for `--gpus N` when it is not already running under
torch.distributed.run: it starts N fresh rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their
environment) before any torch or HIP call in the parent, and relays rank 0's stdout."""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def shard_streams(n_streams: int, world: int, rank: int):
    """stream s -> rank s // ceil(n/world) (contiguous blocks, SURVEY §8e round-robin alternative is equivalent)."""
    per = (n_streams + world - 1) // world
    return list(range(rank * per, min(n_streams, (rank + 1) * per)))


def env_rank():
    """(world, rank, local_rank) from the torch.distributed.run / launch_ranks environment (1, 0, 0 if unset)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, device=None):
    """Join the process group of this rank (env:// rendezvous).  backend "nccl" is RCCL on ROCm."""
    import torch.distributed as dist
    if device is not None:
        dist.init_process_group(backend, device_id=device)
    else:
        dist.init_process_group(backend)
    return dist


def barrier():
    import torch.distributed as dist
    dist.barrier()


def broadcast_arena(tensor, src: int = 0):
    """Broadcast the weight arena (a uint8 tensor aliasing libwmx's device allocation on GPU; a host tensor under
    gloo) from `src`.  The only data-path collective of the job, paid once at start-up."""
    import torch.distributed as dist
    dist.broadcast(tensor, src=src)
    return tensor


class _ArenaView:
    """Zero-copy CUDA-array-interface view of a device allocation (libwmx's weight arena)."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def arena_tensor(model, device):
    """A torch uint8 tensor aliasing the parameter region of the model's weight arena on `device` (no copy;
    wmx_model_arena: the derived copies that follow it are rebuilt per rank by mark_loaded)."""
    import torch
    ptr, nbytes = model.arena()
    return torch.as_tensor(_ArenaView(ptr, nbytes), device=device)


def share_weights(model, rank: int, device, seed: int | None = None, src: int = 0):
    """Make every rank's weights identical: rank `src` initialises (PRNG `seed`, or keeps what is loaded), then ONE RCCL
    broadcast of the arena's parameter region (3.1 GB for large-v3 bf16: the parameters only, not the derived
    row-major / MX-fp8 / 8-bit / folded copies) over xGMI, then every rank derives its copies (mark_loaded).  The only
    data-path collective of the job."""
    import torch
    if rank == src and seed is not None:
        model.init_synthetic(seed)
    view = arena_tensor(model, device)
    torch.cuda.synchronize(device)
    broadcast_arena(view, src=src)
    torch.cuda.synchronize(device)
    model.mark_loaded()
    return view


def max_over_ranks(value: float, device="cpu") -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device="cpu") -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def destroy():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv, script: str, timeout=None) -> int:
    """Start `n` rank processes of `script argv` on this node (127.0.0.1 rendezvous), one per GPU.  Rank 0's stdout
    is relayed (the bench's single JSON line); every rank's stderr passes through.  If a rank fails, the others are
    terminated (a collective would otherwise wait for it forever).  Returns the first non-zero exit code, or 0.
    Must run before this process touches torch / HIP (the children own the GPUs)."""
    import tempfile
    import time
    port = free_port()
    procs = []
    out0 = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL))
    t0, rc = time.time(), 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad or (timeout is not None and time.time() - t0 > timeout):
            rc = bad[0] if bad else 124
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    rc = rc or next((p.returncode for p in procs if p.returncode), 0)
    out0.seek(0)
    sys.stdout.write(out0.read().decode())
    sys.stdout.flush()
    return rc
