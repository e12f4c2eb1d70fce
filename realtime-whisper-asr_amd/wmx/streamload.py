"""BASELINE config 4 on the streaming path: many concurrent synthetic mic streams sharded data-parallel over the GPUs
of one node (stream s -> rank, no cross-stream state, no per-step collective).

Every rank runs the reference's streaming front end for its own streams -- one DynamicVACOnlineASRProcessor per stream
(reference asr_components.py:81-179: the VAD-gated online processor, 1 s online chunks) fed in real-time order, 0.5 s
of audio per tick, and process_iter at that cadence (reference 一键实时识别麦克风.py:1510-1513) -- and batches the due
streams' ASR calls of a tick into ONE transcribe on its GPU (wmx.online.StreamBatcher).  Per stream it records the
committed words (stream, tick, beg, end, text) and the latency of each of its process_iter calls (the wall time of the
batched call it rode in).  At the end the host gathers every rank's records and latencies to rank 0 (the optional
host-side gather of §8e; torch.distributed.all_gather_object over gloo or RCCL, once per run), which reports p50 / p90
over all N x streams.

The streams' audio and VAD tracks depend only on the stream id, so any sharding of the same streams gives the same
per-stream records as one process running them all (tests/test_streamload.py)."""
from __future__ import annotations

import time

import numpy as np

TICK = 8000  # samples per tick: 0.5 s at 16 kHz, the reference loop's process_iter cadence


def stream_audio(stream_id: int, n_samples: int) -> np.ndarray:
    """The synthetic microphone of stream `stream_id` (seeded by the stream id only)."""
    from . import synth
    return synth.speech_like(700 + stream_id, n_samples)


def make_stream(asr, n_samples: int):
    """One mic stream's online processor: the reference's VAD-gated processor with 1 s online chunks, gated by a
    scripted VAD track (speech from the 20th 512-sample window on; Silero weights are not available offline)."""
    from .online import DynamicVACOnlineASRProcessor, ScriptedVAD
    return DynamicVACOnlineASRProcessor(1.0, asr, vad_model=ScriptedVAD([0.0] * 20 + [0.95] * (n_samples // 512 + 2)))


def run_shard(model, asr, stream_ids, seconds: float, make=make_stream, audio=stream_audio, stagger: bool = True,
              final: bool = True):
    """Run this rank's streams tick by tick.  Stream s's audio is fed 0.5 s per tick (odd stream ids one tick late
    when `stagger`: unsynchronised microphones), and every tick the due process_iter calls run as one batched
    transcribe (StreamBatcher.step).  Returns a dict of plain Python values (picklable for the gather):
      records: [(stream, tick, beg, end, text)] committed words, in tick order per stream;
      lat:     [(stream, tick, seconds)] one entry per process_iter that ran the ASR;
      calls:   [(due streams, windows, decode steps, seconds)] per batched call."""
    from .online import StreamBatcher
    ids = list(stream_ids)
    n = int(seconds * 16000)
    audios = {s: audio(s, n) for s in ids}
    streams = [make(asr, n) for _ in ids]
    batcher = StreamBatcher(model, asr)
    cnt = getattr(model, "counters", None) or {"windows": 0, "decode_steps": 0}
    records, lat, calls = [], [], []
    n_ticks = n // TICK + 2
    for k in range(n_ticks):
        for s, p in zip(ids, streams):
            i = (k - (s % 2 if stagger else 0)) * TICK
            if 0 <= i < n:
                p.insert_audio_chunk(audios[s][i: i + TICK])
        due = [s for s, p in zip(ids, streams) if not p.is_currently_final and p.wants_iter()]
        c0 = dict(cnt)
        t0 = time.perf_counter()
        outs = batcher.step(streams)
        dt = time.perf_counter() - t0
        if due:
            calls.append((len(due), cnt.get("windows", 0) - c0.get("windows", 0),
                          cnt.get("decode_steps", 0) - c0.get("decode_steps", 0), dt))
            lat.extend((s, k, dt) for s in due)
        for s, o in zip(ids, outs):
            if o is not None and o[0] is not None:
                records.append((int(s), k, float(o[0]), float(o[1]), str(o[2])))
    if final:  # the end of every stream: flush what LocalAgreement still holds (VACOnlineASRProcessor.finish)
        for s, p in zip(ids, streams):
            o = p.finish()
            if o is not None and o[0] is not None:
                records.append((int(s), n_ticks, float(o[0]), float(o[1]), str(o[2])))
    return {"streams": ids, "records": records, "lat": lat, "calls": calls}


def gather(result, world: int):
    """Every rank's run_shard result on every rank (all_gather_object; world 1: no collective)."""
    if world == 1:
        return [result]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, result)
    return out


def summarize(parts, skip_first_call: bool = True):
    """p50 / p90 of the per-stream process_iter latency over every stream of every rank, and per-call shapes.  The
    first batched call of each rank captures the decode graphs and is left out when it is not the only one."""
    lat, calls, recs, per_rank = [], [], [], []
    for p in parts:
        c = p["calls"]
        first_tick = None
        if skip_first_call and len(c) > 2 and p["lat"]:
            first_tick = min(k for _, k, _ in p["lat"])
            c = c[1:]
        mine = [dt for _, k, dt in p["lat"] if k != first_tick]
        lat.extend(mine)
        # the same first-call exclusion per rank (the per-rank medians were on a different basis)
        per_rank.append(round(1000 * float(np.median(mine)), 2) if mine else None)
        calls.extend(c)
        recs.extend(p["records"])
    return {
        "per_rank_p50_ms": per_rank,
        "streams": sum(len(p["streams"]) for p in parts), "ranks": len(parts),
        "stream_iters": len(lat), "batched_calls": len(calls),
        "p50_ms": round(1000 * float(np.median(lat)), 2) if lat else None,
        "p90_ms": round(1000 * float(np.percentile(lat, 90)), 2) if lat else None,
        "due_streams_per_call": round(float(np.mean([c[0] for c in calls])), 2) if calls else None,
        "windows_per_call": round(float(np.mean([c[1] for c in calls])), 2) if calls else None,
        "decode_steps_per_call": round(float(np.mean([c[2] for c in calls])), 1) if calls else None,
        "tick_busy": round(float(np.mean([c[3] for c in calls])) / (TICK / 16000.0), 3) if calls else None,
        "committed": len(recs),
    }
