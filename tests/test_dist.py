"""World-size-2 gloo test of the multi-GPU plumbing used by bench.py (wmx.dist): stream sharding covers every
stream exactly once, the weight-arena broadcast makes every rank bit-identical to rank 0, and the timing reduction
takes the max over ranks.  (On MI355X the same calls run over RCCL / xGMI.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from wmx import dist as D
    mine = D.shard_streams(13, world, rank)
    got = [None] * world
    dist.all_gather_object(got, mine)
    arena = torch.arange(4096, dtype=torch.int32).to(torch.uint8) if rank == 0 else torch.zeros(4096, dtype=torch.uint8)
    D.broadcast_arena(arena, src=0)
    t = D.max_over_ranks(1.5 + rank)
    s = D.sum_over_ranks(float(len(mine)))
    out[rank] = (got, bool(torch.equal(arena, torch.arange(4096, dtype=torch.int32).to(torch.uint8))), t, s)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharding_broadcast_and_max(world):
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        shards, arena_ok, tmax, total = out[r]
        flat = sorted(x for sh in shards for x in sh)
        assert flat == list(range(13))
        assert arena_ok
        assert tmax == 1.5 + world - 1
        assert total == 13.0
