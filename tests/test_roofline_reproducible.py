"""the bench line's headline roofline is reproducible from the committed rocprofv3 summary.
tools/roofline_from_stats.py recomputes the packed-GEMM family's fraction of HBM peak from a `--kernel-trace --stats`
kernel_stats CSV (average durations x launches per layer-step) and the line's algorithmic bytes; the final build's
default and 16-window fp8 lines must agree with their own rocprofv3 runs within 6 % (the traced run decodes in the
tracer-induced slow mode, so its kernels run slightly longer than the line's)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles", "r05z")


@pytest.mark.parametrize("stats,line", [("kernel_stats_bf16.csv", "bench_default.json"),
                                        ("kernel_stats_fp8_b16.csv", "bench_fp8_b16.json")])
def test_line_frac_matches_rocprof_summary(stats, line):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_from_stats.py"),
                          os.path.join(P, stats), os.path.join(P, line)], capture_output=True, text=True, check=True)
    r = json.loads(out.stdout)
    assert r["layer_step_us"] > 0 and len(r["instantiations"]) >= 3, r
    assert 0.94 <= r["agreement"] <= 1.06, (r["frac"], r["line_frac"], r["agreement"])
