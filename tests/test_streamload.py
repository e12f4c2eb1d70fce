"""Config 4's streaming path sharded over ranks (wmx.streamload), on the CPU with a fake ASR engine:
world-size-2 gloo ranks each run their shard of the mic streams (DynamicVACOnlineASRProcessor per stream at the
reference cadence, one batched ASR call per tick through StreamBatcher), rank 0 gathers (stream, tick, beg, end,
text) and the latencies, and the gathered records equal one process running every stream."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


class _Word:
    def __init__(self, s, e, w, p=0.9):
        self.start, self.end, self.word, self.probability = s, e, w, p


class _Seg:
    def __init__(self, words):
        self.words, self.end, self.start = words, words[-1].end, words[0].start


class FakeModel:
    """Stands in for wmx.transcribe.WhisperModel.transcribe_batch: one word per 0.5 s of each buffer, its text a
    deterministic function of that half-second's samples (so results depend on the stream's audio only, never on
    which other streams share the batch)."""
    max_batch, groups = 64, 1

    def __init__(self):
        self.counters = {"windows": 0, "engine_calls": 0, "decode_steps": 0}
        self.batches = []

    def transcribe_batch(self, audios, prompts=None, language=None, task="transcribe", beam_size=None, temperature=0.0,
                         best_of=5, **kw):
        self.batches.append(len(audios))
        self.counters["windows"] += len(audios)
        self.counters["engine_calls"] += 1
        self.counters["decode_steps"] += 10 * len(audios)
        out = []
        for a in audios:
            words = []
            for i in range(len(a) // 8000):
                h = int(np.abs(a[i * 8000:(i + 1) * 8000]).sum() * 7) % 1000
                words.append(_Word(i * 0.5, i * 0.5 + 0.4, f" w{h}"))
            out.append([_Seg(words[j:j + 4]) for j in range(0, len(words), 4)])
        return out


class FakeASRView:
    sep = ""
    transcribe_kargs = {"beam_size": 5}
    original_language = None

    def ts_words(self, segments):
        return [(w.start, w.end, w.word) for s in segments for w in s.words]

    def segments_end_ts(self, segments):
        return [s.end for s in segments]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_streams, seconds, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from wmx import dist as D
    from wmx import streamload as SL
    mine = D.shard_streams(n_streams, world, rank)
    res = SL.run_shard(FakeModel(), FakeASRView(), mine, seconds)
    parts = SL.gather(res, world)
    if rank == 0:
        out["parts"] = parts
        out["summary"] = SL.summarize(parts)
    dist.destroy_process_group()


def _by_stream(records):
    d = {}
    for s, k, b, e, t in records:
        d.setdefault(s, []).append((k, round(b, 6), round(e, 6), t))
    return d


@pytest.mark.parametrize("world", [2])
def test_sharded_streams_gather_equals_one_process(world):
    from wmx import streamload as SL
    n_streams, seconds = 5, 6.0
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n_streams, seconds, out), nprocs=world, join=True)
    parts = out["parts"]
    assert [p["streams"] for p in parts] == [[0, 1, 2], [3, 4]]  # contiguous shards, every stream once
    gathered = [r for p in parts for r in p["records"]]
    single = SL.run_shard(FakeModel(), FakeASRView(), range(n_streams), seconds)
    assert gathered, "the streams must commit words"
    assert _by_stream(gathered) == _by_stream(single["records"])
    for s, recs in _by_stream(gathered).items():  # committed words are time-ordered per stream
        ends = [e for _, _, e, _ in recs]
        assert ends == sorted(ends), s
    summ = out["summary"]
    assert summ["streams"] == n_streams and summ["ranks"] == world
    assert summ["stream_iters"] > 0 and summ["p50_ms"] is not None and summ["p90_ms"] >= summ["p50_ms"]
    # every rank's latencies are per stream iteration: each due stream of a tick appears once
    for p in parts:
        ticks = [(s, k) for s, k, _ in p["lat"]]
        assert len(ticks) == len(set(ticks))
        assert {s for s, _ in ticks} <= set(p["streams"])


def test_run_shard_batches_due_streams_per_tick():
    """One StreamBatcher call per tick carries every due stream of the shard (the staggered streams are due on
    alternate ticks once their buffers pass the 1 s online chunk)."""
    from wmx import streamload as SL
    m = FakeModel()
    res = SL.run_shard(m, FakeASRView(), range(4), 5.0)
    assert m.batches and max(m.batches) >= 2
    assert sum(c[0] for c in res["calls"]) == len(res["lat"])
