#!/usr/bin/env python3
"""Benchmark of the MI355X streaming-Whisper hot path (BASELINE.json metric: real-time factor + p50 chunk
latency, Whisper large-v3 30 s @ 16 kHz, 1/2/4/8 GPUs).

Workload (BASELINE.json configs[2]/[3]): Whisper large-v3 dims, bf16, synthetic weights (build-owned PRNG; no
checkpoint is reachable offline), B concurrent synthetic 30 s mic streams per GPU; one step = one batched
transcribe call over the B windows = log-mel -> encoder -> cross K/V -> language detection -> prompt prefill ->
beam-5 decode (hipGraph per step) -> word alignment (alignment forward + DTW), inputs resident in HBM.
Streams are independent (data parallel): stream s runs on rank s // B; the only collective is the RCCL broadcast
of the weight arena from rank 0 at start-up ("scaling": "weak").

value = audio seconds processed by all ranks / max-over-ranks wall time  (x real time = 1 / RTF).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# HIP hardware queues per process (read at HIP initialisation, so before anything touches the GPU): the decoding
# context groups, the model stream and torch's streams exceed HIP's default of 4; runs fall into a slower decode mode
# (544-563 vs 538 ms per call) less often with 8 queues (2 of 14 runs vs 3 of 7, profiles/r02p_hwq_ab/ and
# r02q_kernarg_ab/).  An explicit setting from the caller wins.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "realtime-whisper-asr_amd"))
sys.path.insert(0, ROOT)

METRIC = "real-time factor + p50 chunk latency, Whisper large-v3 30s@16kHz, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0
MFMA_BF16_PEAK_TFLOPS = 2500.0
MFMA_FP8_PEAK_TFLOPS = 5000.0  # MI355X dense fp8 / MX-fp8 (no sparsity)
MAX_CLOCK_MHZ = 2400.0  # MI355X_MICROARCH.md: the clock the dense peaks are quoted at
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector = FP32 matrix peak, spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_JSON_OUT = None


def emit(obj):
    """The one JSON line, on the real stdout (native libraries' stdout chatter is redirected to stderr)."""
    out = _JSON_OUT or sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def quiet_stdout():
    """Point fd 1 at stderr so RCCL / gloo / HIP messages printed by native code cannot interleave with the JSON
    line; keep a private handle on the original stdout for emit()."""
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="large-v3")
    p.add_argument("--batch", type=int, default=8, help="concurrent 30 s streams per GPU")
    p.add_argument("--groups", type=int, default=2, help="concurrent decoding contexts the streams are split over")
    p.add_argument("--beam", type=int, default=5)
    p.add_argument("--max-new-tokens", type=int, default=224)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "fp8", "int8"],
                   help="fp8: BASELINE config 5 (encoder projections on the MX-fp8 MFMA, decoder and logits "
                        "projections on 8-bit weights, fp8 cross-K/V images; activations bf16); int8: the reference's "
                        "int8_float16 (CTranslate2's int8 grid for the decoder and logits projections, f16 activations)")
    p.add_argument("--task", default="transcribe", choices=["transcribe", "translate"])
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU rehearsal of the launch / rendezvous / broadcast / max-over-ranks plumbing (gloo, no GPU)")
    p.add_argument("--no-stream", action="store_true", help="skip the per-stream process_iter latency lines")
    return p.parse_args()


# WMX_* variables a measured line may run under: documented knobs that select a configuration the line then reports
# (each is recorded in the line's "env").  Anything else named WMX_* is a timing-only or removed experiment switch
# (WMX_ABLATE dropped launches from the decode step, results wrong by construction; WMX_PHASE_PROBE / _DUMP, WMX_FOLD,
# WMX_MLP_FUSED, WMX_REDLN_FUSED, WMX_XATTN_* were measured-slower variants, removed in round 6): the bench refuses
# to print a line under one.
BENCH_ENV_KNOBS = {
    "WMX_LIB": "library path (A/B builds)",
    "WMX_ROOT": "repository root (test harness)",
    "WMX_LOCKSTEP": "0: the context groups' decode loops start independently",
    "WMX_LOCKSTEP_CHUNKS": "0: lockstep barrier at the decode start only",
    "WMX_STREAM_GROUPS": "contexts per batched stream call (stream_load line)",
    "WMX_DEC_MIXED": "0: the fast decode step (three reduce_ln launches per layer) instead of the default mixed step",
    "WMX_DEC_FP8": "0: keep the fp8 model's decode on 16-bit weights",
    "WMX_ENC_FOLD": "0: encoder LayerNorms as their own launches",
    "WMX_XQ_FUSED": "0: the cross-q projection as its own split-K launch",
    "WMX_CROSS_CHUNK": "decode cross-attention key chunk",
    "WMX_SILERO_WEIGHTS": "Silero v5 safetensors path (VAD line)",
}


def check_env():
    """The WMX_* environment of this run: returns it (recorded in the line); exits with status 2 and no line when a
    variable outside BENCH_ENV_KNOBS is set."""
    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith("WMX_")}
    bad = [k for k in env if k not in BENCH_ENV_KNOBS]
    if bad:
        log(f"bench.py: refusing to measure under timing-only / unknown switches {bad}: a line measured under them "
            f"is not the product path (documented knobs: {sorted(BENCH_ENV_KNOBS)})")
        sys.exit(2)
    return env


def held_clock(run, device=0, ms=120.0, n=8):
    """The shader clock the chip holds while `run()` executes (the clock in the encoder field):
    n single-wave workgroups of libwmx's clock probe (wmx_debug_clock_start / _result, include/wmx_diag.h) sleep on
    a stream of their own for `ms` of the 100 MHz constant clock, started just before `run`, each reporting
    d(s_memtime) / d(s_memrealtime) x 100 MHz on its XCD.  Returns (run's result, {median / min / max MHz, ...})."""
    import ctypes as C
    from wmx._lib import lib, check
    check(lib.wmx_debug_clock_start(device, ms, n))
    try:
        res = run()
    finally:
        buf = (C.c_float * n)()
        check(lib.wmx_debug_clock_result(buf, n))
    v = sorted(float(x) for x in buf)
    return res, {"median_mhz": round(v[n // 2], 1), "min_mhz": round(v[0], 1), "max_mhz": round(v[-1], 1),
                 "window_ms": ms, "probes": n,
                 "how": "in-kernel d(s_memtime)/d(s_memrealtime) x 100 MHz of n sleeping waves (one per XCD) over "
                        "the first window_ms of the passes (MI355X_MICROARCH.md 'DVFS give-back' item 6)"}


def _cpu_sample(W, d, args, steps_done, n_text):
    """One bounded sample of the oracle on this host: one 30 s window, log-mel + encoder + language detection +
    prompt prefill + 4 beam decode steps (per-step time extrapolated to the GPU run's step count) + the word
    alignment pass (alignment forward over n_text tokens + DTW).  Returns (seconds per window, stage log)."""
    from oracle import whisper_np as O
    from wmx import synth
    audio = synth.speech_like(10_000, 480000)
    tm = {}
    t = time.perf_counter()
    mel = O.logmel_segment(audio, d.n_mels)
    tm["mel"] = time.perf_counter() - t
    t = time.perf_counter()
    enc = O.encoder(W, d, mel)
    tm["enc"] = time.perf_counter() - t
    t = time.perf_counter()
    lang, _ = O.detect_language(W, d, enc)
    tm["lang"] = time.perf_counter() - t
    sp = O.special_tokens(d.n_vocab)
    t = time.perf_counter()
    cache = O.DecoderCache(W, d, enc)
    O.decoder_forward(W, d, O.sot_sequence(sp, lang, "transcribe"), cache)
    tm["prefill"] = time.perf_counter() - t
    caches = [cache.copy() for _ in range(args.beam)]
    n_dec = 4
    t = time.perf_counter()
    for s in range(n_dec):
        for c in caches:
            O.decoder_forward(W, d, [sp.timestamp_begin + s], c)
    tm["step"] = (time.perf_counter() - t) / n_dec
    t = time.perf_counter()
    O.find_alignment(W, d, enc, lang, "transcribe", [1000 + (i % 5000) for i in range(n_text)], 3000)
    tm["align"] = time.perf_counter() - t
    total = tm["mel"] + tm["enc"] + tm["lang"] + tm["prefill"] + tm["step"] * max(steps_done, 1) + tm["align"]
    return total, tm


def cpu_baseline(model, args, steps_done, n_text):
    """The oracle (numpy fp32 restatement, oracle/whisper_np.py) timed on this host's cores as the proxy for the
    reference CPU path (faster-whisper / CT2 int8 is not installed: SURVEY §8d), at CT2's default 4 intra-op
    threads and at every core of the affinity mask (BLAS threads set with threadpoolctl)."""
    from oracle import whisper_np as O
    from threadpoolctl import threadpool_limits

    d = O.DIMS[args.model] if args.model in O.DIMS else None
    # BASELINE.md §4 states the host core count from the affinity mask.  On the GPU box that mask lists the whole
    # machine (256) while this job's CPU share is 16 (the pool's per-GPU share, exported as OMP_NUM_THREADS; a cgroup
    # quota when one is set): 256 BLAS threads on 16 CPUs time oversubscription, not the CPU path, so the all-cores
    # leg runs at the smallest of the three and all three are reported
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0")) or None
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = max(1, int(int(q) / int(per))) if q != "max" else None
    except (OSError, ValueError):
        pass
    cores = min(x for x in (affinity, omp, quota) if x)
    t0 = time.perf_counter()
    W = {}
    for name, shape, _, _ in O.tensor_specs(d):
        W[name] = model.get_tensor(name, shape)
    W["encoder.embed_positions.weight"] = O.sinusoids(1500, d.n_audio_state)
    log(f"[cpu] weights read back in {time.perf_counter() - t0:.1f}s")
    out = {}
    for threads in (4, cores):
        with threadpool_limits(limits=threads):
            total, tm = _cpu_sample(W, d, args, steps_done, n_text)
        log(f"[cpu] {threads} threads: " + " ".join(f"{k} {v:.3f}s" for k, v in tm.items()) +
            f" (step x {steps_done}) -> {total:.1f}s per 30 s window")
        out[threads] = (total, tm)
    total4 = out[4][0]
    totalc = out[cores][0]
    return {"value": round(30.0 / total4, 4), "unit": "x_realtime", "cores": 4, "kind": "proxy",
            "all_cores": {"value": round(30.0 / totalc, 4), "cores": cores},
            "host": {"sched_getaffinity": affinity, "OMP_NUM_THREADS": omp, "cgroup_cpu_quota": quota,
                     "cores_note": "all_cores = min(affinity, OMP_NUM_THREADS, cgroup quota): the CPUs this job "
                                   "may use on the box (16 of the machine's 256 per GPU), not the machine's count"},
            "sample": f"1 x 30 s window of {args.model} through the numpy fp32 oracle (faster-whisper/CT2 absent: "
                      f"proxy): log-mel + encoder + language detect + prefill + 4 beam-{args.beam} decode steps "
                      f"(per-step time extrapolated to the GPU run's {steps_done} steps) + word alignment over "
                      f"{n_text} tokens; value at 4 BLAS threads (CT2's default), all_cores at {cores}"}


def stream_latency(name, dtype, seconds, cadence_s, max_new_tokens, vac):
    """Per-stream p50 of one process_iter -> transcribe call, through the drop-in adapter and the
    streaming processors: `vac` = config 2 (DynamicVACOnlineASRProcessor, 1 s online chunks, 640-sample feed,
    scripted VAD track), else EnhancedOnlineASRProcessor with process_iter every `cadence_s` (一键.py:1510)."""
    from wmx import synth
    from wmx.asr import MI355XWhisperASR
    from wmx.online import DynamicVACOnlineASRProcessor, EnhancedOnlineASRProcessor, ScriptedVAD
    asr = MI355XWhisperASR(lan="auto", modelsize=name, device="cuda", compute_type=dtype,
                           transcribe_kwargs={"beam_size": 5}, max_new_tokens=max_new_tokens)
    lat, cost = [], []
    inner = asr.transcribe
    cnt = asr.model.counters

    def timed(audio, init_prompt=""):
        c0 = dict(cnt)
        t0 = time.perf_counter()
        out = inner(audio, init_prompt=init_prompt)
        lat.append(time.perf_counter() - t0)
        cost.append((cnt["windows"] - c0["windows"], cnt["decode_steps"] - c0["decode_steps"], len(audio) / 16000))
        return out

    asr.transcribe = timed
    audio = synth.speech_like(77, int(seconds * 16000))
    tick = []
    if vac:
        from wmx.vad import SileroVAD
        n_win = len(audio) // 512

        class DeviceSileroScripted:
            """The device Silero network runs on every 512-sample window (its cost is in the VAC tick), but its
            synthetic weights cannot detect speech, so the gate follows a scripted track."""

            def __init__(self, probs):
                self.net, self.track = SileroVAD(), ScriptedVAD(probs)

            def reset_states(self):
                self.net.reset_states()
                self.track.reset_states()

            def __call__(self, x, sr=16000):
                self.net(x, sr)
                return self.track(x, sr)

        proc = DynamicVACOnlineASRProcessor(
            1.0, asr, vad_model=DeviceSileroScripted([0.0] * 30 + [0.95] * (n_win - 30)))
        feed, every = 640, 1
    else:
        proc = EnhancedOnlineASRProcessor(asr, buffer_trimming=("segment", 15), agreement_n=3)
        feed, every = int(cadence_s * 16000), 1
    for i in range(0, len(audio), feed):
        t0 = time.perf_counter()
        proc.insert_audio_chunk(audio[i: i + feed])
        tick.append(time.perf_counter() - t0)
        if (i // feed) % every == 0:
            proc.process_iter()
    if len(lat) > 2:  # the first call captures the decode graph
        lat, cost = lat[1:], cost[1:]
    return {"model": f"whisper-{name}", "dtype": dtype, "calls": len(lat),
            "p50_ms": round(1000 * float(np.median(lat)), 2) if lat else None,
            "p90_ms": round(1000 * float(np.percentile(lat, 90)), 2) if lat else None,
            # what one call is made of: 30 s windows decoded (the seek loop continues after a window that does not end
            # on a timestamp pair; random weights never emit EOT, so every window decodes max_new_tokens) and decode
            # steps, per call, and the buffer length the calls saw
            "windows_per_call": round(float(np.mean([c[0] for c in cost])), 2) if cost else None,
            "decode_steps_per_call": round(float(np.mean([c[1] for c in cost])), 1) if cost else None,
            "buffer_s_mean": round(float(np.mean([c[2] for c in cost])), 2) if cost else None,
            "insert_chunk_p50_ms": round(1000 * float(np.median(tick)), 3),
            "feed": "VAC, 640-sample chunks, 1 s online chunks, device Silero VAD per window (synthetic weights; "
                    "gate on a scripted track)" if vac else f"process_iter every {cadence_s} s", "audio_s": seconds,
            "max_new_tokens": max_new_tokens, "beam": 5}


def stream_load(name, dtype, n_per_gpu, seconds, max_new_tokens, world=1, rank=0):
    """Per-stream chunk latency UNDER LOAD (BASELINE's second number at config 4: 64 streams over 8 GPUs = 8 per GPU),
    on the streaming path sharded over ranks (wmx.streamload): n_per_gpu x world synthetic mic streams,
    stream s on rank shard_streams(...), each a DynamicVACOnlineASRProcessor (reference asr_components.py:81-179; 1 s
    online chunks, scripted VAD track) fed in real-time order 0.5 s per tick (the reference loop calls process_iter
    every 0.5 s, 一键实时识别麦克风.py:1510-1513), odd streams one tick late (unsynchronised mics).  Every tick, a
    rank's due process_iter calls run as ONE batched transcribe on its GPU (StreamBatcher); a due stream's latency is
    that call's wall time.  Rank 0 gathers every rank's (stream, tick, beg, end, text) records and latencies
    (all_gather_object, once) and reports p50 / p90 over all streams, windows and decode steps per batched call, and
    the GPU busy fraction of the tick budget (mean call time / 0.5 s; > 1 cannot keep up in real time)."""
    from wmx import dist as D
    from wmx import streamload as SL
    from wmx.asr import MI355XWhisperASR
    asr = MI355XWhisperASR(lan="auto", modelsize=name, device="cuda", compute_type=dtype,
                           transcribe_kwargs={"beam_size": 5}, max_new_tokens=max_new_tokens)
    model = asr.model
    mine = D.shard_streams(n_per_gpu * world, world, rank)
    model.max_batch = max(1, len(mine))
    model._ctx.clear()
    # one context per batched call; WMX_STREAM_GROUPS=2 splits a tick's due windows over two contexts decoding in step
    # (WhisperModel.groups, wmx_ctx_set_lockstep): 4 windows per call measured 515-519 against 511-513 ms p50, so
    # the split pays only from larger batches (the 8-window bench line)
    model.groups = int(os.environ.get("WMX_STREAM_GROUPS", "1"))
    res = SL.run_shard(model, asr, mine, seconds)
    parts = SL.gather(res, world)
    out = SL.summarize(parts)
    out.update({"model": f"whisper-{name}", "dtype": dtype, "audio_s_per_stream": seconds,
                "streams_per_gpu": n_per_gpu,
                "feed": "VAC (1 s online chunks, scripted VAD track), 0.5 s per tick, streams staggered by one tick; "
                        "one batched transcribe per tick per rank over its due streams (StreamBatcher); streams sharded "
                        "over ranks (wmx.dist.shard_streams), records and latencies gathered to rank 0",
                "context_groups": model.groups, "max_new_tokens": max_new_tokens, "beam": 5})
    return out


def vad_bench(streams):
    """Silero VAD v5 on device (wmx_vad_process, synthetic weights): wall time per call, host audio in, probabilities
    out, for one VAC tick of this GPU's streams (one 512-sample window each) and a 16-window backlog of 64 streams."""
    from wmx import synth, vad
    res = []
    for S_, W_ in ((streams, 1), (64, 16)):
        eng = vad.SileroVADEngine(max_streams=S_, max_windows=W_)
        chunk = {s: synth.speech_like(50 + s, 512 * W_).astype(np.float32) for s in range(S_)}
        for _ in range(5):
            eng.process(chunk)
        n = 50
        t0 = time.perf_counter()
        for _ in range(n):
            eng.process(chunk)
        us = (time.perf_counter() - t0) / n * 1e6
        eng.close()
        res.append({"streams": S_, "windows_per_stream": W_, "us_per_call": round(us, 1),
                    "windows_per_s": round(S_ * W_ / (us * 1e-6), 1)})
    return {"calls": res, "note": "wall clock per wmx_vad_process (H2D + 2 launches + D2H + sync), synthetic weights"}


def dry_run(args):
    """The multi-rank plumbing of main() without a GPU: gloo rendezvous, the arena broadcast, barrier-bracketed
    timed steps, max over ranks, one JSON line from rank 0 (tests/test_bench_launch.py drives it at world 2)."""
    from wmx import dist as D
    import torch
    world, rank, _ = D.env_rank()
    if world > 1:
        D.init("gloo")
    arena = (torch.arange(1 << 16, dtype=torch.int32) % 251).to(torch.uint8)
    if rank != 0:
        arena.zero_()
    if world > 1:
        D.broadcast_arena(arena, src=0)
    ok = bool(torch.equal(arena, (torch.arange(1 << 16, dtype=torch.int32) % 251).to(torch.uint8)))
    x = np.random.default_rng(rank).standard_normal(480000).astype(np.float32)

    def step():  # a fixed synthetic host workload standing in for one transcribe call
        return float(np.abs(np.fft.rfft(x.reshape(-1, 400), axis=-1)).sum())

    for _ in range(args.warmup):
        step()
    if world > 1:
        D.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        D.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = D.max_over_ranks(elapsed)
        ranks = int(D.sum_over_ranks(1.0))
        arena_ok = int(D.sum_over_ranks(float(ok))) == world
    else:
        ranks, arena_ok = 1, ok
    if rank == 0:
        value = 30.0 * args.batch * world * args.steps / elapsed
        emit({"metric": METRIC, "value": round(value, 3), "unit": "x_realtime (audio s / wall s, all GPUs)",
              "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
              "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
              "scaling": "weak", "vs_baseline": None, "dtype": "f32",
              "data": "dry run: launch / rendezvous / broadcast plumbing only, host FFT stand-in step",
              "config": {"workload": "dry-run", "parallelism": f"dp{world} (independent streams)"},
              "ranks_reporting": ranks, "arena_broadcast_ok": arena_ok})
    D.destroy()


def main():
    args = parse()
    wmx_env = check_env()
    from wmx import dist as D
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` outside torch.distributed.run: start N rank processes here, before any torch / HIP
        # call in this process, and relay rank 0's JSON line
        sys.exit(D.launch_ranks(args.gpus, sys.argv[1:], os.path.abspath(__file__)))
    quiet_stdout()
    if args.dry_run:
        return dry_run(args)
    world, rank, local = D.env_rank()
    if world != args.gpus:
        log(f"[rank {rank}] note: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)")
    dist = None
    # torch (plumbing only: RCCL + the resident input buffer) must bring up its HIP runtime before libwmx is
    # loaded, so the process holds ONE libamdhip64.so.7 and device pointers are shared.
    import torch
    torch.cuda.set_device(local)
    torch.zeros(1, device=f"cuda:{local}")
    if world > 1:
        dist = D.init("nccl", torch.device("cuda", local))  # RCCL
    from wmx import engine, synth

    dt = {"bf16": "bfloat16", "f16": "float16", "fp8": "float8", "int8": "int8_float16"}[args.dtype]
    model = engine.Model(args.model, local, dt)
    t = time.time()
    if world > 1:
        D.share_weights(model, rank, torch.device("cuda", local), seed=args.seed)  # RCCL over xGMI
    else:
        model.init_synthetic(args.seed)
    log(f"[rank {rank}] weights ready in {time.time() - t:.2f}s ({model.n_params() / 1e9:.2f} B params)")

    B = args.batch
    G = args.groups
    assert B % G == 0, "--batch must be a multiple of --groups"
    Bg = B // G
    heads = engine.ALIGNMENT_HEADS.get(args.model)
    # G decoding contexts (each its own HIP stream and captured decode graph) share the weights; their window
    # groups run concurrently, so one group's kernel boundaries and latency-bound phases overlap the other's work
    ctxs = [engine.Context(model, max_batch=Bg, beam_size=args.beam, max_new_tokens=args.max_new_tokens, task=args.task,
                           language=None, word_timestamps=True, alignment_heads=heads, use_graph=not args.no_graph)
            for _ in range(G)]
    ctx = ctxs[0]
    # the groups' decode loops start together (wmx_ctx_set_lockstep): in step they share each layer's weight reads
    # through the caches; started a few layers apart they do not, and the call runs ~5 % slower (the
    # slow decode mode).  WMX_LOCKSTEP=0 turns it off (A/B runs)
    lockstep = G > 1 and os.environ.get("WMX_LOCKSTEP", "1") != "0"
    if lockstep:
        for c in ctxs:
            c.set_lockstep(1, G)
    # synthetic 30 s streams, resident in HBM before the timed region
    audio = np.stack([synth.speech_like(rank * B + i, 480000) for i in range(B)])
    pcm = torch.from_numpy(audio).to(f"cuda:{local}")
    lens = np.full(Bg, 480000, np.int64)
    torch.cuda.synchronize()
    pool = None
    if G > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=G)  # ctypes drops the GIL inside libwmx calls

    def step():
        if G == 1:
            return ctx.transcribe_device(pcm.data_ptr(), 480000, lens)
        futs = [pool.submit(c.transcribe_device, pcm.data_ptr() + g * Bg * 480000 * 4, 480000, lens)
                for g, c in enumerate(ctxs)]
        out = []
        for f in futs:
            out.extend(f.result())
        return out

    # in-situ probes captured into each context's decode-step graph: device-clock start / end of the six packed
    # projection GEMMs and the cross attention of the middle decoder layer, at every step of the timed decode loops
    probe_layer = model.dims.n_text_layer // 2
    for g, c in enumerate(ctxs):
        c.set_probe(True, probe_layer)
    for _ in range(args.warmup):
        step()
    if dist is not None:
        D.barrier()
    torch.cuda.synchronize()
    lat = []
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        ts = time.perf_counter()
        res = step()
        lat.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    if dist is not None:
        D.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = D.max_over_ranks(elapsed, device=f"cuda:{local}")
    stages = ctx.stage_ms()
    steps_done = ctx.last_steps()
    n_tok = [len(r.tokens) for r in res]
    log(f"[rank {rank}] stage ms (logmel, enc, xkv, lang, prefill, decode, align): "
        f"{[round(s, 2) for s in stages]}  decode steps {steps_done}  tokens/window {n_tok}")

    audio_s = 30.0 * B * world * args.steps
    value = audio_s / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    p50 = 1000.0 * float(np.median(lat))

    # roofline of the dominant kernel family.  achieved = ALGORITHMIC bytes / launch duration; the duration is
    # measured in situ over the timed region by device-clock probes on every launch of layer `probe_layer` (and the
    # previous layer's last one), every decode step, both context groups: a launch's duration = its last workgroup
    # end minus its predecessor's -- dispatch + execution, the per-kernel span rocprofv3 reports (the rocprofv3 trace
    # of this bench is recomputed by tools/roofline_from_profile.py into profiles/).  Beside it: the execution-only
    # workgroup span of the same launches, and 20 back-to-back replays of each launch alone (HIP events on the
    # context stream, after the timed region)
    def gather(events):
        agg = {}
        for c in ctxs:
            for k, (ms_k, n_k, by_k) in c.probe_launches(e2e=events).items():
                a = agg.setdefault(k, [0.0, 0, by_k])
                a[0] += ms_k * n_k
                a[1] += n_k
        return {k: (v[0] / v[1] if v[1] else 0.0, v[1], v[2]) for k, v in agg.items()}
    evs = gather(True)      # end-to-end: dispatch + execution (rocprofv3's per-kernel span)
    insitu = gather(False)  # first-workgroup-start .. last-workgroup-end
    replay_id = {"dec_qkv": "dec_qkv", "dec_out": "dec_proj", "dec_cross_q": "dec_proj", "dec_cross_out": "dec_proj",
                 "dec_fc1": "dec_fc1", "dec_fc2": "dec_fc2", "cross_attn": "cross_attn"}
    if evs["dec_cross_q"][1] == 0 and evs["cross_attn"][1] > 0:  # cross-q projection fused into the cross attention
        del replay_id["dec_cross_q"]
    replay_cache = {}
    for k, rid in replay_id.items():
        if rid not in replay_cache:
            replay_cache[rid] = ctx.bench_kernel(rid, Bg, iters=20)
    replay = {k: (replay_cache[rid][0], replay_cache[rid][1]) for k, rid in replay_id.items()}
    use_ev = all(evs[k][1] > 0 for k in replay_id)
    launch = {k: ((evs[k][0], evs[k][2]) if use_ev else replay[k]) for k in replay_id}
    fams = {"gemm_packed_kernel": [k for k in launch if k.startswith("dec_")], "dec_cross_attn_kernel": ["cross_attn"]}
    fam_ms = {f: sum(launch[k][0] for k in ks) for f, ks in fams.items()}  # per layer-step, one group
    dom = max(fam_ms, key=fam_ms.get)
    ms_e2e = fam_ms[dom]
    by = sum(launch[k][1] for k in fams[dom])
    # the duration basis of `frac`: the in-situ END-TO-END time of each launch (its last
    # workgroup's end minus its predecessor's: dispatch + execution, what rocprofv3's kernel trace reports as the
    # kernel's duration), so the headline can be recomputed from the committed rocprofv3 kernel_stats summary.  The
    # execution span (first workgroup start .. last workgroup end, device clock) is kept as a labelled secondary
    # figure: with two context groups in step each launch runs beside the other group's same launch, and the span of
    # one group's launch divides the bytes by a window the GPU also spent on the other's (it overstates, r04: 0.215
    # on the span basis against 0.164 end to end and 0.153 from rocprofv3)
    span_ms = sum(insitu[k][0] for k in fams[dom]) if all(insitu.get(k, (0, 0))[1] for k in fams[dom]) else 0.0
    contended = False
    ms = ms_e2e
    ach = by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "frac_basis": ("end-to-end in situ (dispatch + execution of each launch, rocprofv3's kernel duration; "
                           f"{G} context group(s), every launch of layer {probe_layer} in every timed decode step)"
                           if use_ev else "isolated replay")}
    roof["frac_end_to_end"] = round(by / (ms_e2e * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if ms_e2e > 0 else None
    roof["frac_span"] = round(by / (span_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if span_ms > 0 else None
    roof["frac_span_note"] = ("secondary: execution span of one group's launches (first workgroup start .. last end); "
                              "overstates when the groups' same launches run at once and share the weight reads")
    rep_ms = sum(replay[k][0] for k in fams[dom])
    roof["frac_isolated_replay"] = round(by / (rep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if rep_ms > 0 else None
    # HBM traffic per launch from the committed rocprofv3 PMC passes (tools/pmc_traffic.py: FETCH_SIZE x2 +
    # WRITE_SIZE, separate passes) of the same launches replayed alone at this context's batch
    for tag in ("r05", "r04", "r03", "r02", "r01g"):
        pmc = os.path.join(ROOT, "profiles", f"{tag}_pmc_traffic.json")
        if not os.path.exists(pmc):
            continue
        recs = json.load(open(pmc))
        # (entries keyed launch@windows-per-group; the fp8 decode's launches carry a /fp8 suffix)
        sfx = {"fp8": "/fp8", "int8": "/int8"}.get(args.dtype, "")
        got = [recs.get(f"{replay_id[k]}@{Bg}{sfx}") for k in fams[dom]]
        if all(got):
            tb = sum(g["traffic_bytes"] for g in got)
            roof["traffic"] = round(tb / 1e9 / (ms * 1e-3), 1)
            roof["traffic_bytes_per_layer_step"] = tb
            roof["traffic_source"] = f"profiles/{tag}_pmc_traffic.json (FETCH_SIZE x2 + WRITE_SIZE, separate passes)"
            break
    roof["kernel"] = dom
    roof["measured"] = (f"in situ over the timed region: device-clock end of each launch of layer {probe_layer} minus "
                        f"its predecessor's, every decode step, both groups, {sum(evs[k][1] for k in fams[dom])} "
                        f"launch samples" if use_ev else
                        "HIP events around 20 back-to-back replays of each launch (wmx_ctx_bench_kernel)")
    def _dur(k):
        return insitu[k][0] if contended else launch[k][0]
    roof["launches"] = {k: {"us": round(1000 * _dur(k), 2), "bytes": launch[k][1],
                            "gbs": round(launch[k][1] / (_dur(k) * 1e-3) / 1e9, 1)} for k in fams[dom]}
    roof["algorithmic_bytes_per_layer_step"] = by
    roof["layer_step_ms"] = round(ms, 4)
    roof["family_ms_per_layer_step"] = {f: round(v, 4) for f, v in fam_ms.items()}
    roof["replayed_us"] = {k: round(1000 * replay[k][0], 2) for k in fams[dom]}
    # every probed launch of the layer, end to end (the whole layer-step chain of one group, in launch order)
    roof["layer_e2e_us"] = {k: round(1000 * v[0], 2) for k, v in evs.items() if v[1] and k != "prev_layer_last"}
    # the decode step form (wmx_runtime.hip): "mixed" (default for 16-bit models since round 6: the out / cross-out
    # projections unsplit with the residual add and row statistics in their epilogue, one reduce_ln per layer) or
    # "fast" (three reduce_ln launches per layer).  The mixed step moves the residual + LayerNorm work of two
    # reduce_ln launches INTO two of the family's launches, so `frac` (family bytes / family time) is not comparable
    # across the forms; frac_projection_chain divides the same bytes by the family's time plus every reduce_ln launch
    # of the layer, which is.  (replayed_us / frac_isolated_replay / traffic are of the split-K launch forms.)
    red_keys = [k for k in ("reduce_ln_out", "reduce_ln_cross_out", "reduce_ln_fc2") if evs.get(k, (0, 0))[1]]
    roof["decode_step"] = "fast" if "reduce_ln_out" in red_keys else "mixed"
    chain_ms = ms_e2e + sum(evs[k][0] for k in red_keys)
    roof["frac_projection_chain"] = round(by / (chain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if chain_ms > 0 else None
    roof["layer_span_us"] = {k: round(1000 * v[0], 2) for k, v in insitu.items() if v[1] and k != "prev_layer_last"}
    span = sum(insitu[k][0] for k in fams[dom])
    roof["wg_span"] = {"what": f"device-clock span first workgroup start .. last workgroup end, layer {probe_layer}, "
                               f"every timed decode step, both groups", "samples": sum(insitu[k][1] for k in fams[dom]),
                       "us": {k: round(1000 * insitu[k][0], 2) for k in fams[dom]},
                       "achieved_gbs": round(by / (span * 1e-3) / 1e9, 1) if span > 0 else None}
    # decode mode (about 1 run in 4 fell into a mode 3-5 % slower, in which the packed GEMMs and the
    # reduce + LayerNorm launches run 10-25 % longer while the cross attention runs faster): the in-situ ratio of the
    # cross attention to the rest of the GEMM / reduce chain, calibrated on the r02 runs (fast 0.365-0.372, slow
    # 0.324-0.334; profiles/r02p_hwq_ab/, r02q_kernarg_ab/)
    chain = [k for k in ("dec_qkv", "dec_out", "dec_cross_out", "dec_fc1", "dec_fc2", "reduce_ln_out",
                         "reduce_ln_cross_out", "reduce_ln_fc2") if evs.get(k, (0, 0))[1]]
    decode_mode = None
    if chain and evs.get("cross_attn", (0, 0))[1]:
        ratio = evs["cross_attn"][0] / sum(evs[k][0] for k in chain)
        decode_mode = {"mode": "fast" if ratio >= 0.35 else "slow", "cross_to_chain_ratio": round(ratio, 4),
                       "rule": "cross attention / (packed GEMMs + reduce_ln) in situ >= 0.35 -> fast"}
        if args.dtype in ("fp8", "int8"):  # 8-bit weights halve the GEMMs' bytes (fp8 also the cross attention's): the
            decode_mode["mode"] = "n/a (rule calibrated on the bf16 decode)"  # bf16 calibration does not hold
        # per context group: the slow mode can hit one group alone, and the call takes the
        # slower group's time; each group's decode stage and its own ratio
        per_group = []
        for c in ctxs:
            ev_g = c.probe_launches(e2e=True)
            ch = [k for k in chain if ev_g.get(k, (0, 0))[1]]
            r_g = (ev_g["cross_attn"][0] / sum(ev_g[k][0] for k in ch)
                   if ch and ev_g.get("cross_attn", (0, 0))[1] else None)
            per_group.append({"decode_stage_ms": round(c.stage_ms()[5], 2),
                              "cross_to_chain_ratio": round(r_g, 4) if r_g is not None else None})
        decode_mode["groups"] = per_group
        log(f"[rank {rank}] decode mode: {decode_mode}")
    # the other named stages: the log-mel front end (north_star: HBM GB/s of the mel path) and the self attention,
    # replayed alone with HIP events on the context stream
    kern_stats = {}
    for k in ("logmel", "self_attn", "reduce_ln"):
        kern_stats[k] = ctx.bench_kernel(k, Bg, iters=20)
    lm_ms, lm_by, lm_fl = kern_stats["logmel"]
    logmel = {"windows": Bg, "us": round(1000 * lm_ms, 1), "bytes": lm_by,
              "achieved_gbs": round(lm_by / (lm_ms * 1e-3) / 1e9, 1),
              "frac_hbm": round(lm_by / (lm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "tflops_f32": round(lm_fl / (lm_ms * 1e-3) / 1e12, 2),
              "frac_f32_peak": round(lm_fl / (lm_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFLOPS, 4),
              "bound": "latency / f32 vector ALU",
              "note": "isolated replay, HIP events (raw + finalize launches); the windowed real DFT is a two-pass "
                      "20 x 20 Cooley-Tukey transform on the vector ALUs (~54 kFLOP per frame), the audio, partial "
                      "spectra, power and filterbank in LDS; HBM would allow ~2 us per window"}
    # encoder MFMA utilisation (north_star: >= 40 % in the encoder): one whole encoder pass over a context's
    # windows, isolated (HIP events), and the in-situ encoder stage of the timed region (all groups concurrent)
    # three 3-pass averages (the clock the chip holds after the decode-heavy timed region varies by a few %): the
    # MEDIAN is reported (the best of three biased the utilisation upward), all three beside it
    def med3(c, b):
        runs = sorted(c.bench_kernel("encoder", b, iters=3) for _ in range(3))
        return runs[1], [round(r[0], 3) for r in runs]
    (e_ms, _, e_fl), e_runs = med3(ctx, Bg)
    e_tf = e_fl / (e_ms * 1e-3) / 1e12
    insitu_tf = G * e_fl / (stages[1] * 1e-3) / 1e12 if stages[1] > 0 else None
    # the same pass over the whole per-GPU batch (B windows in one launch sequence), in a scratch context
    e_ms_b, e_fl_b = e_ms, e_fl
    if G > 1:
        scratch = engine.Context(model, max_batch=B, beam_size=1, max_new_tokens=8, word_timestamps=False,
                                 use_graph=False)
        ((e_ms_b, _, e_fl_b), e_runs_b), sclk = held_clock(lambda: med3(scratch, B), device=local)
        scratch.close()
    else:
        ((e_ms_b, _, e_fl_b), e_runs_b), sclk = held_clock(lambda: med3(ctx, B), device=local)
    e_tf_b = e_fl_b / (e_ms_b * 1e-3) / 1e12
    encoder = {"windows": Bg, "gflop_per_window": round(e_fl / Bg / 1e9, 1), "isolated_ms": round(e_ms, 2),
               "isolated_tflops": round(e_tf, 1), "isolated_mfma_util": round(e_tf / MFMA_BF16_PEAK_TFLOPS, 4),
               "isolated_passes_ms": e_runs,
               "isolated_gpu_batch": {"windows": B, "ms": round(e_ms_b, 2), "tflops": round(e_tf_b, 1),
                                      "mfma_util": round(e_tf_b / MFMA_BF16_PEAK_TFLOPS, 4),
                                      "passes_ms": e_runs_b,
                                      "best_mfma_util": round(e_fl_b / (min(e_runs_b) * 1e-3) / 1e12 /
                                                              MFMA_BF16_PEAK_TFLOPS, 4),
                                      "held_clock": sclk,
                                      "mfma_util_at_held_clock": round(e_tf_b / (MFMA_BF16_PEAK_TFLOPS *
                                                                       sclk["median_mhz"] / MAX_CLOCK_MHZ), 4)},
               "insitu_stage_ms": round(stages[1], 2),
               "insitu_tflops": round(insitu_tf, 1) if insitu_tf else None,
               "insitu_mfma_util": round(insitu_tf / MFMA_BF16_PEAK_TFLOPS, 4) if insitu_tf else None,
               "peak_tflops": MFMA_BF16_PEAK_TFLOPS,
               "timing": "isolated: HIP events, median of three 3-pass averages after one warm pass (all three "
                         "listed)",
               "note": ("fp8: the projections run on the MX-fp8 MFMA (5 PF dense peak), attention and convs bf16; "
                        "mfma_util above is against the bf16 peak, mfma_util_vs_dtype_peak against each op's own "
                        "peak" if args.dtype == "fp8" else "bf16 MFMA")}
    if args.dtype == "fp8":
        # the pass's ideal time with the projections at the fp8 peak and the attention / convs at the bf16 peak, over
        # the measured time (quote the fp8 encoder against the fp8 peak)
        md = model.dims
        da, La, T = md.n_audio_state, md.n_audio_layer, 1500.0
        proj = 24.0 * La * T * da * da * B
        rest = e_fl_b - proj
        ideal_s = proj / (MFMA_FP8_PEAK_TFLOPS * 1e12) + rest / (MFMA_BF16_PEAK_TFLOPS * 1e12)
        encoder["isolated_gpu_batch"]["mfma_util_vs_dtype_peak"] = round(ideal_s / (e_ms_b * 1e-3), 4)
        encoder["isolated_gpu_batch"]["projection_flop_share"] = round(proj / e_fl_b, 4)
    log(f"[rank {rank}] encoder: {encoder}")
    log(f"[rank {rank}] in-situ span us/launch (layer {probe_layer}): " +
        ", ".join(f"{k}={1000 * v[0]:.2f}" for k, v in insitu.items() if v[1]))
    log(f"[rank {rank}] in-situ end-to-end us/launch: " + ", ".join(f"{k}={1000 * v[0]:.2f}" for k, v in evs.items() if v[1]))
    log(f"[rank {rank}] replayed us/launch: " + ", ".join(f"{k}={1000 * v[0]:.2f}" for k, v in replay.items()))
    log(f"[rank {rank}] replayed kernel us/launch: " + ", ".join(f"{k}={1000 * v[0]:.2f}" for k, v in kern_stats.items()))

    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "x_realtime (audio s / wall s, all GPUs)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2),
        "p50_chunk_latency_ms": round(p50, 2),
        "rtf": round(1.0 / value * world, 6),
        "chunks_per_s": round(B * world * args.steps / elapsed, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded speech-like 30 s audio; build-owned PRNG weights of the named architecture)",
        "config": {"workload": f"whisper-{args.model} {args.task}, {B} x 30 s windows per GPU, beam {args.beam}, "
                               f"word_timestamps, language auto-detect, max_new_tokens {args.max_new_tokens}",
                   "model": f"whisper-{args.model}", "global_batch": B * world, "seq_len": 480000,
                   "parallelism": f"dp{world} (independent streams)", "decode_steps": steps_done,
                   "use_graph": not args.no_graph, "context_groups": G,
                   **({"int8_rule": "int8 weights (CTranslate2's grid and row scales) x 16-bit activations; "
                                    "CTranslate2's dynamic int8 activation quantisation is not applied "
                                    "(INTEGRATION.md)"} if args.dtype == "int8" else {})},
        "stage_ms": [round(s, 2) for s in stages],
        "env": wmx_env,
        "decode_mode": decode_mode,
        "lockstep": lockstep,
        "roofline": roof,
        "encoder": encoder,
        "logmel": logmel,
        "self_attn_us": round(1000 * kern_stats["self_attn"][0], 2),
        "reduce_ln_us": round(1000 * kern_stats["reduce_ln"][0], 2),
    }
    try:  # reported beside the headline, never the target
        out["vad"] = vad_bench(B)
        log(f"[rank {rank}] silero vad: {out['vad']}")
    except Exception as e:
        log(f"[vad] failed: {e!r}")
    if rank == 0 and world == 1 and not args.no_stream:
        # per-stream p50 of process_iter -> transcribe, next to the batched call's latency above
        out["stream_latency"] = []
        for cfg in ((args.model, dt, 8.0, 0.5, args.max_new_tokens, False), ("base", "float16", 12.0, 1.0, 64, True)):
            try:
                out["stream_latency"].append(stream_latency(*cfg))
            except Exception as e:  # reported, never the target
                log(f"[stream] {cfg[0]} failed: {e!r}")
        log(f"[rank {rank}] stream latency: {out['stream_latency']}")
    if not args.no_stream:
        # the same per-stream latency under load, config 4's streaming path: B streams per GPU (64 streams / 8 GPUs),
        # sharded over every rank, gathered to rank 0 (every rank takes part: the gather is a collective)
        try:
            out["stream_load"] = stream_load(args.model, dt, B, 12.0, args.max_new_tokens, world, rank)
            log(f"[rank {rank}] stream load: {out['stream_load']}")
        except Exception as e:  # reported, never the target
            log(f"[stream load] failed: {e!r}")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            n_text = max(1, int(np.mean([sum(t < 50257 for t in r.tokens) for r in res])))
            out["cpu_baseline"] = cpu_baseline(model, args, steps_done, n_text)
        except Exception as e:  # the baseline is reported, never the target
            log(f"[cpu] baseline failed: {e!r}")
            out["cpu_baseline"] = None
    if rank == 0:
        emit(out)
    D.destroy()


if __name__ == "__main__":
    main()
