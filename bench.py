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

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "realtime-whisper-asr_amd"))
sys.path.insert(0, ROOT)

METRIC = "real-time factor + p50 chunk latency, Whisper large-v3 30s@16kHz, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0
MFMA_BF16_PEAK_TFLOPS = 2500.0


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
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "fp8"],
                   help="fp8: BASELINE config 5 (encoder projections on the MX-fp8 MFMA, the rest bf16)")
    p.add_argument("--task", default="transcribe", choices=["transcribe", "translate"])
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU rehearsal of the launch / rendezvous / broadcast / max-over-ranks plumbing (gloo, no GPU)")
    p.add_argument("--roofline-kernel", default="auto",
                   choices=["auto", "cross_attn", "enc_fc1", "enc_attn", "logmel", "dec_fc1", "self_attn"])
    return p.parse_args()


class _ArenaView:
    """Zero-copy torch view of the library's weight arena (for the RCCL broadcast)."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def cpu_baseline(model, args, steps_done):
    """The oracle (numpy fp32 restatement, oracle/whisper_np.py) timed on this host on a bounded sample:
    one 30 s window: log-mel + encoder + language detection + prompt prefill + 4 beam decode steps; the per-step
    time is extrapolated to the same number of decode steps the GPU run executed."""
    from oracle import whisper_np as O
    from wmx import synth

    d = O.DIMS[args.model] if args.model in O.DIMS else None
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    t0 = time.perf_counter()
    W = {}
    for name, shape, _, _ in O.tensor_specs(d):
        W[name] = model.get_tensor(name, shape)
    W["encoder.embed_positions.weight"] = O.sinusoids(1500, d.n_audio_state)
    t_load = time.perf_counter() - t0
    audio = synth.speech_like(10_000, 480000)
    t = time.perf_counter()
    mel = O.logmel_segment(audio, d.n_mels)
    t_mel = time.perf_counter() - t
    t = time.perf_counter()
    enc = O.encoder(W, d, mel)
    t_enc = time.perf_counter() - t
    t = time.perf_counter()
    lang, _ = O.detect_language(W, d, enc)
    t_lang = time.perf_counter() - t
    sp = O.special_tokens(d.n_vocab)
    t = time.perf_counter()
    cache = O.DecoderCache(W, d, enc)
    O.decoder_forward(W, d, O.sot_sequence(sp, lang, "transcribe"), cache)
    t_pre = time.perf_counter() - t
    caches = [cache.copy() for _ in range(args.beam)]
    n_dec = 4
    t = time.perf_counter()
    for s in range(n_dec):
        for c in caches:
            O.decoder_forward(W, d, [sp.timestamp_begin + s], c)
    t_step = (time.perf_counter() - t) / n_dec
    total = t_mel + t_enc + t_lang + t_pre + t_step * max(steps_done, 1)
    log(f"[cpu] load {t_load:.1f}s mel {t_mel:.3f}s enc {t_enc:.2f}s lang {t_lang:.2f}s prefill {t_pre:.2f}s "
        f"step {t_step:.3f}s x {steps_done} -> {total:.1f}s per 30 s window")
    return {"value": round(30.0 / total, 4), "unit": "x_realtime", "cores": cores, "kind": "port",
            "sample": f"1 x 30 s window of {args.model} (numpy fp32 oracle): log-mel + encoder + language detect + "
                      f"prefill + {n_dec} beam-{args.beam} decode steps timed, per-step time extrapolated to "
                      f"{steps_done} steps; word alignment not included"}


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

    dt = {"bf16": "bfloat16", "f16": "float16", "fp8": "float8"}[args.dtype]
    model = engine.Model(args.model, local, dt)
    t = time.time()
    if world > 1:
        if rank == 0:
            model.init_synthetic(args.seed)
        ptr, nbytes = model.arena()
        view = torch.as_tensor(_ArenaView(ptr, nbytes), device=f"cuda:{local}")
        torch.cuda.synchronize()
        D.broadcast_arena(view, src=0)  # RCCL over xGMI: the only collective of the job
        torch.cuda.synchronize()
        model.mark_loaded()
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

    # in-situ probe: HIP events captured into each context's decode-step graph around the cross-attention launch
    # of the middle decoder layer, sampled once per 8-step replay chunk during the timed decode loops
    for c in ctxs:
        c.set_probe("cross_attn", model.dims.n_text_layer // 2)
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

    # roofline of the dominant kernel, measured live with HIP events on the context stream
    per_step_ms = {}
    kern_stats = {}
    R = B * args.beam
    counts = {  # launches per transcribe step (each context group launches its own, over Bg windows)
        "cross_attn": G * steps_done * model.dims.n_text_layer,
        "self_attn": G * steps_done * model.dims.n_text_layer,
        "dec_fc1": G * steps_done * model.dims.n_text_layer,
        "enc_fc1": G * model.dims.n_audio_layer,
        "enc_attn": G * model.dims.n_audio_layer,
        "logmel": G,
    }
    for k in counts:
        log(f"[rank {rank}] timing kernel {k}")
        ms, by, fl = ctx.bench_kernel(k, Bg, iters=20)
        kern_stats[k] = (ms, by, fl)
        per_step_ms[k] = ms * counts[k]
    dom = max(per_step_ms, key=per_step_ms.get) if args.roofline_kernel == "auto" else args.roofline_kernel
    ms, by, fl = kern_stats[dom]
    measured = "isolated replay (wmx_ctx_bench_kernel, HIP events, 20 launches)"
    if dom == "cross_attn":
        # the in-situ launches of the timed region (all context groups running concurrently)
        st = [c.probe_stats() for c in ctxs]
        n = sum(x[1] for x in st)
        if n:
            ms = sum(x[0] * x[1] for x in st) / n
            by = st[0][2]
            measured = f"in-situ, timed region: {n} sampled launches (layer {model.dims.n_text_layer // 2})"
    if dom in ("enc_fc1", "enc_attn"):
        ach = fl / (ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": None}
    else:
        ach = by / (ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None}
    # HBM traffic per launch from the committed rocprofv3 PMC passes (tools/pmc_traffic.py) at this launch's batch
    pmc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01g_pmc_traffic.json")
    if os.path.exists(pmc):
        rec = json.load(open(pmc)).get(f"{dom}@{Bg}")
        if rec and roof["unit"] == "GB/s":
            roof["traffic"] = round(rec["traffic_bytes"] / 1e9 / (ms * 1e-3), 1)
            roof["traffic_bytes_per_launch"] = rec["traffic_bytes"]
            roof["traffic_source"] = "profiles/r01g_pmc_traffic.json (FETCH_SIZE x2 + WRITE_SIZE, separate passes)"
    roof["measured"] = measured
    roof["kernel"] = dom
    roof["launch_ms"] = round(ms, 4)
    roof["algorithmic_per_launch"] = {"bytes": by, "flops": fl}
    # encoder MFMA utilisation (north_star: >= 40 % in the encoder): one whole encoder pass over a context's
    # windows, isolated (HIP events), and the in-situ encoder stage of the timed region (all groups concurrent)
    e_ms, _, e_fl = ctx.bench_kernel("encoder", Bg, iters=3)
    e_tf = e_fl / (e_ms * 1e-3) / 1e12
    insitu_tf = G * e_fl / (stages[1] * 1e-3) / 1e12 if stages[1] > 0 else None
    # the same pass over the whole per-GPU batch (B windows in one launch sequence), in a scratch context
    e_ms_b, e_fl_b = e_ms, e_fl
    if G > 1:
        scratch = engine.Context(model, max_batch=B, beam_size=1, max_new_tokens=8, word_timestamps=False,
                                 use_graph=False)
        e_ms_b, _, e_fl_b = scratch.bench_kernel("encoder", B, iters=3)
        scratch.close()
    e_tf_b = e_fl_b / (e_ms_b * 1e-3) / 1e12
    encoder = {"windows": Bg, "gflop_per_window": round(e_fl / Bg / 1e9, 1), "isolated_ms": round(e_ms, 2),
               "isolated_tflops": round(e_tf, 1), "isolated_mfma_util": round(e_tf / MFMA_BF16_PEAK_TFLOPS, 4),
               "isolated_gpu_batch": {"windows": B, "ms": round(e_ms_b, 2), "tflops": round(e_tf_b, 1),
                                      "mfma_util": round(e_tf_b / MFMA_BF16_PEAK_TFLOPS, 4)},
               "insitu_stage_ms": round(stages[1], 2),
               "insitu_tflops": round(insitu_tf, 1) if insitu_tf else None,
               "insitu_mfma_util": round(insitu_tf / MFMA_BF16_PEAK_TFLOPS, 4) if insitu_tf else None,
               "peak_tflops": MFMA_BF16_PEAK_TFLOPS,
               "note": ("fp8: the projections run on the MX-fp8 MFMA (5 PF dense peak), attention and convs bf16; "
                        "utilisation quoted against the bf16 peak" if args.dtype == "fp8" else "bf16 MFMA")}
    log(f"[rank {rank}] encoder: {encoder}")
    log(f"[rank {rank}] kernel ms/launch: " + ", ".join(f"{k}={v[0]:.4f}" for k, v in kern_stats.items()))
    log(f"[rank {rank}] est. ms per transcribe step: " + ", ".join(f"{k}={v:.1f}" for k, v in per_step_ms.items()))

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
                   "use_graph": not args.no_graph, "context_groups": G},
        "stage_ms": [round(s, 2) for s in stages],
        "roofline": roof,
        "encoder": encoder,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(model, args, steps_done)
        except Exception as e:  # the baseline is reported, never the target
            log(f"[cpu] baseline failed: {e!r}")
            out["cpu_baseline"] = None
    if rank == 0:
        emit(out)
    D.destroy()


if __name__ == "__main__":
    main()
