"""The relative phase of the bench's two context groups, call by call (diagnostic for the slow decode mode, DESIGN.md
§7): the default bench workload (large-v3 bf16, 8 windows as 2 groups of 4, beam 5, 224 tokens, word timestamps),
the decode-step probes on layer 16, and per call: each group's decode stage, its mean step period, and the offset of
group 1's cross attention start from group 0's at the same step, modulo the layer period.

  python tools/phase_probe.py [--calls 4] [--out file.json]"""
import argparse
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "realtime-whisper-asr_amd"))

import torch  # noqa: E402

torch.cuda.init()
from wmx import engine, synth  # noqa: E402

CROSS = engine.Context.PROBE_LAUNCHES.index("cross_attn")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--out", default=None)
    ap.add_argument("--lockstep", type=int, default=0, help="1: the groups' decode loops start together")
    ap.add_argument("--phase-offset-us", type=float, default=0.0, help="group g idles g x this before its decode loop")
    args = ap.parse_args()
    torch.zeros(1, device="cuda:0")
    m = engine.Model("large-v3", 0, "bfloat16")
    m.init_synthetic(1)
    heads = engine.ALIGNMENT_HEADS.get("large-v3")
    B, G = 8, 2
    Bg = B // G
    ctxs = [engine.Context(m, max_batch=Bg, beam_size=5, max_new_tokens=224, task="transcribe", language=None,
                           word_timestamps=True, alignment_heads=heads) for _ in range(G)]
    audio = np.stack([synth.speech_like(i, 480000) for i in range(B)])
    pcm = torch.from_numpy(audio).to("cuda:0")
    lens = np.full(Bg, 480000, np.int64)
    for c in ctxs:
        c.set_probe(True, 16)
        if args.lockstep:
            c.set_lockstep(7, G)
    for g, c in enumerate(ctxs):
        c.set_phase_offset(g * args.phase_offset_us)
    pool = ThreadPoolExecutor(max_workers=G)
    rows = []
    for call in range(args.calls + 1):  # call 0 = warm-up
        futs = [pool.submit(c.transcribe_device, pcm.data_ptr() + g * Bg * 480000 * 4, 480000, lens)
                for g, c in enumerate(ctxs)]
        for f in futs:
            f.result()
        torch.cuda.synchronize()
        if call == 0:
            continue
        t = [c.probe_ticks() for c in ctxs]
        khz = t[0][1]
        st = [tk[0][:, CROSS, 0].astype(np.float64) / khz * 1e3 for tk in t]  # cross attention starts, us
        n = min(len(st[0]), len(st[1]))
        ok = (st[0][:n] > 0) & (st[1][:n] > 0)
        per = [float(np.median(np.diff(s[s > 0]))) for s in st]  # step period, us
        layer_us = float(np.mean(per)) / 33.0  # 32 layers + the step's tail (logits, selection, beam) ~ one layer
        d = (st[1][:n] - st[0][:n])[ok]
        ph = np.mod(d, layer_us) / layer_us
        hist = np.histogram(ph, bins=10, range=(0, 1))[0].tolist()
        # the 8-step graph chunks: the step period across a chunk boundary (host read-back of n_done + the next
        # chunk's graph launch) against the period inside a chunk
        bnd = []
        for s_ in st:
            s_ = s_[s_ > 0]
            dd = np.diff(s_)
            at = np.arange(1, len(s_)) % 8 == 0
            bnd.append([round(float(np.median(dd[~at])), 1), round(float(np.median(dd[at])), 1) if at.any() else None])
        row = {"call": call, "period_inside_vs_across_chunk_us": bnd, "decode_ms": [round(c.stage_ms()[5], 2) for c in ctxs],
               "step_period_us": [round(p, 1) for p in per], "layer_period_us": round(layer_us, 2),
               "offset_us_median": round(float(np.median(d)), 1), "offset_us_drift": round(float(d[-1] - d[0]), 1),
               "offset_us_min_max": [round(float(d.min()), 1), round(float(d.max()), 1)],
               "offset_us_by_chunk": [round(float(np.median(d[i:i + 8])), 1) for i in range(0, len(d), 8)],
               "phase_median": round(float(np.median(ph)), 3), "phase_hist10": hist}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
