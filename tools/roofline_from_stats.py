#!/usr/bin/env python3
"""The bench's headline roofline recomputed from a rocprofv3 --stats kernel summary: the
packed-GEMM family of one decoder layer-step = the decode's gemm_packed_kernel instantiations weighted by how many
launches of each a layer-step makes (the d x d projections out and cross-out share one instantiation: 2 per layer),
their AVERAGE rocprofv3 durations summed, the bench line's algorithmic bytes per layer-step divided by that sum.

usage: python tools/roofline_from_stats.py <kernel_stats.csv> <bench line .json> [n_layers]
Prints the per-instantiation averages and the frac next to the line's own roofline.frac."""
import csv
import json
import sys


def main(stats, line, n_layers=32):
    rows = list(csv.DictReader(open(stats)))
    d = json.loads([x for x in open(line) if x.strip().startswith("{")][-1])
    roof = d["roofline"]
    by = roof["algorithmic_bytes_per_layer_step"]
    steps = d["config"]["decode_steps"] * (d["steps"] + d["warmup"])  # decode steps of the profiled calls, per group
    groups = d["config"].get("context_groups", 1)
    packed = [r for r in rows if "gemm_packed_kernel" in r["Name"]]
    # the decode's instantiations: the most-called ones; a layer-step launches ~ calls / (layers x steps x groups)
    # of each (the profiled run also holds warm-up calls, language detection and prefill, so round to the nearest)
    per = []
    for r in sorted(packed, key=lambda r: -int(r["Calls"])):
        k = int(r["Calls"]) / max(1, n_layers * steps * groups)
        if k >= 0.5:
            per.append((r["Name"].split(">(")[0] + ">", round(k), float(r["AverageNs"]) / 1000.0, int(r["Calls"])))
    us = sum(n * a for _, n, a, _ in per)
    ach = by / (us * 1e-6) / 1e9
    # the projection chain (comparable across the fast and mixed decode steps: the mixed step folds two reduce_ln
    # launches' work into two of the family's launches): the family plus the layer-step's reduce_ln4 launches
    red = [r for r in rows if "reduce_ln4_kernel" in r["Name"]]
    red_us = sum(round(int(r["Calls"]) / max(1, n_layers * steps * groups)) * float(r["AverageNs"]) / 1000.0
                 for r in red if int(r["Calls"]) / max(1, n_layers * steps * groups) >= 0.5)
    out = {"kernel_stats": stats, "bench_line": line, "algorithmic_bytes_per_layer_step": by,
           "instantiations": [{"name": nm, "per_layer_step": n, "avg_us": round(a, 3), "calls": c}
                              for nm, n, a, c in per],
           "layer_step_us": round(us, 3), "achieved_gbs": round(ach, 1), "frac": round(ach / 8000.0, 4),
           "line_frac": roof["frac"], "line_basis": roof.get("frac_basis"),
           "agreement": round(roof["frac"] / (ach / 8000.0), 4) if us > 0 else None,
           "reduce_ln_us_per_layer_step": round(red_us, 3),
           "frac_projection_chain": round(by / ((us + red_us) * 1e-6) / 1e9 / 8000.0, 4) if us + red_us > 0 else None,
           "line_frac_projection_chain": roof.get("frac_projection_chain")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 32)
