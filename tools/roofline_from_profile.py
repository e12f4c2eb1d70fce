"""Roofline of the decode-step kernels recomputed from a rocprofv3 --kernel-trace CSV (the cross-check of
bench.py's in-situ `roofline`).

Every decode step on a queue is  embed_ln, then per decoder layer  [packed qkv, self attention, packed out,
reduce_ln, (packed cross-q,) cross attention, packed cross-out, reduce_ln, packed fc1, packed fc2, reduce_ln]
(no cross-q launch when the cross attention projects its own queries, the default: detected from the count),
then the packed logits GEMM and the selection kernels (wmx_runtime.hip dec_step_fast / run_step).  The packed
GEMM launches of a step are labelled by their position; durations are averaged per label over every decode step
of every queue; algorithmic bytes per launch are those bench.py uses (weights + 16-bit activations in and out).

  python tools/roofline_from_profile.py run_kernel_trace.csv --layers 32 --d 1280 --rows 20 --windows 4
"""
import argparse
import collections
import csv
import json

PROJ6 = ("dec_qkv", "dec_out", "dec_cross_q", "dec_cross_out", "dec_fc1", "dec_fc2")
PROJ5 = ("dec_qkv", "dec_out", "dec_cross_out", "dec_fc1", "dec_fc2")  # cross-q fused into the cross attention


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--d", type=int, default=1280)
    ap.add_argument("--rows", type=int, default=20, help="decode rows per context (windows x beam)")
    ap.add_argument("--windows", type=int, default=4, help="windows per context")
    ap.add_argument("--peak", type=float, default=8000.0)
    args = ap.parse_args()
    byq = collections.defaultdict(list)
    for r in csv.DictReader(open(args.trace)):
        byq[r.get("Queue_Id", r.get("Stream_Id"))].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    dur = collections.defaultdict(list)
    steps = 0
    L = args.layers
    # packed launches per layer: count them in the first complete step of any queue
    P = 6
    for q, ks in byq.items():
        ks.sort()
        at = [i for i, k in enumerate(ks) if "embed_ln_kernel" in k[2]]
        if len(at) >= 2:
            n_p = sum("gemm_packed_kernel" in k[2] for k in ks[at[0]:at[1]])
            P = 5 if n_p == 5 * L + 1 else 6
            break
    PROJ = PROJ5 if P == 5 else PROJ6
    for q, ks in byq.items():
        ks.sort()
        i, n = 0, len(ks)
        while i < n:
            if "embed_ln_kernel" not in ks[i][2]:
                i += 1
                continue
            steps += 1
            i += 1
            p = 0
            while i < n and "embed_ln_kernel" not in ks[i][2] and "logmel" not in ks[i][2]:
                s, e, name = ks[i]
                if "gemm_packed_kernel" in name:
                    if p < P * L:
                        dur[PROJ[p % P]].append(e - s)
                    elif p == P * L:
                        dur["logits"].append(e - s)
                    p += 1
                elif "dec_cross_attn_kernel" in name:
                    dur["cross_attn"].append(e - s)
                elif "dec_self_attn_kernel" in name:
                    dur["self_attn"].append(e - s)
                elif "reduce_ln" in name:
                    dur["reduce_ln"].append(e - s)
                if p > P * L:
                    break
                i += 1
    d, R, B = args.d, args.rows, args.windows

    def proj(nn, k):
        return nn * k * 2 + R * k * 2 + R * nn * 2

    algo = {"dec_qkv": proj(3 * d, d), "dec_out": proj(d, d), "dec_cross_q": proj(d, d), "dec_cross_out": proj(d, d),
            "dec_fc1": proj(4 * d, d), "dec_fc2": proj(d, 4 * d), "cross_attn": B * 1500 * 2 * d * 2 + 2 * R * d * 2
            + (d * d * 2 + R * d * 2 if P == 5 else 0)}
    out = {"decode_steps_seen": steps, "launches": {}}
    for k, v in sorted(dur.items()):
        us = sum(v) / len(v) / 1000.0
        rec = {"n": len(v), "avg_us": round(us, 3)}
        if k in algo:
            rec["bytes"] = algo[k]
            rec["gbs"] = round(algo[k] / (us * 1e-6) / 1e9, 1)
        out["launches"][k] = rec
    fam = [k for k in PROJ if k in out["launches"]]
    if fam:
        t = sum(out["launches"][k]["avg_us"] for k in fam)
        b = sum(algo[k] for k in fam)
        out["gemm_packed_kernel"] = {"us_per_layer_step": round(t, 3), "bytes": b,
                                     "achieved_gbs": round(b / (t * 1e-6) / 1e9, 1),
                                     "frac": round(b / (t * 1e-6) / 1e9 / args.peak, 4)}
    if "cross_attn" in out["launches"]:
        c = out["launches"]["cross_attn"]
        out["dec_cross_attn_kernel"] = {"achieved_gbs": c["gbs"], "frac": round(c["gbs"] / args.peak, 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
