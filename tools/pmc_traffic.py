"""HBM traffic per launch of the hot-path kernels from rocprofv3 PMC counters.

Each counter gets its own rocprofv3 pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), over
`tools/kbench.py <kernel>` replaying one kernel.  FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: on gfx950 it
reports half the bytes of a wide coalesced streaming read); WRITE_SIZE is taken as is.  Both are in KB.
Writes a JSON summary (default profiles/r01_pmc_traffic.json) that bench.py reports as roofline.traffic.

Run on the GPU box:  python tools/pmc_traffic.py cross_attn dec_fc1
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernel-name substrings of the timed launch (the helper launches of a replay are excluded)
MATCH = {
    "cross_attn": "dec_cross_attn_kernel",
    "self_attn": "dec_self_attn_kernel",
    "dec_fc1": "gemm_packed_kernel",
    "enc_fc1": "gemm256_kernel",
    "enc_attn": "enc_attn_kernel",
    "logmel": "logmel_raw_kernel",
    "dec_qkv": "gemm_packed_kernel",
    "dec_proj": "gemm_packed_kernel",
    "dec_fc2": "gemm_packed_kernel",
    "reduce_ln": "reduce_ln",
}


def run_pass(kernel, counter, out_dir, batch, dtype="bfloat16"):
    d = os.path.join(out_dir, f"{kernel}_{batch}_{dtype}_{counter}")
    cmd = ["rocprofv3", "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.join(ROOT, "tools", "kbench.py"), kernel, "--iters", "10", "--batch", str(batch),
           "--dtype", dtype]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=300)
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if MATCH[kernel] in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise RuntimeError(f"no {counter} samples for {kernel}")
    vals = vals[1:] if len(vals) > 1 else vals  # drop the warm-up launch
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels", nargs="+")
    ap.add_argument("--batch", type=int, nargs="+", default=[4, 8], help="windows per launch")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_pmc_traffic.json"))
    ap.add_argument("--dtype", nargs="+", default=["bfloat16"],
                    help="model dtypes; float8 entries are keyed kernel@batch/fp8 (the 8-bit weights / fp8 images), "
                         "int8_float16 ones kernel@batch/int8 (CTranslate2's int8 grid)")
    ap.add_argument("--work", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    args = ap.parse_args()
    res = {}
    if os.path.exists(args.out):  # passes are added to an existing summary (one GPU call per dtype / batch set)
        res = json.load(open(args.out))
    for dt in args.dtype:
        sfx = "/fp8" if dt == "float8" else "/int8" if dt.startswith("int8") else ""
        for k in args.kernels:
            for b in args.batch:
                fetch_kb, n1 = run_pass(k, "FETCH_SIZE", args.work, b, dt)
                write_kb, n2 = run_pass(k, "WRITE_SIZE", args.work, b, dt)
                res[f"{k}@{b}{sfx}"] = {"batch": b, "dtype": dt, "fetch_bytes": 2.0 * fetch_kb * 1024,
                                        "write_bytes": write_kb * 1024,
                                        "traffic_bytes": 2.0 * fetch_kb * 1024 + write_kb * 1024,
                                        "launches": min(n1, n2),
                                        "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; KB = 1024 B"}
                print(k, b, dt, json.dumps(res[f"{k}@{b}{sfx}"]), flush=True)
                with open(args.out, "w") as f:  # written as it goes: a later pass that fails keeps the earlier ones
                    json.dump(res, f, indent=1)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
