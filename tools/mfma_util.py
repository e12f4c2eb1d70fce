"""MFMA-pipe utilisation and held clock per kernel from one rocprofv3 counter pass.

  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d <dir> -o pmc -- python tools/encprof.py bfloat16
  python tools/mfma_util.py <dir>/run_results.db (or a run_counter_collection.csv) [kernel-substring ...]

Per dispatch:
  * active cycles per XCD = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the counter over the 8 XCDs, MI355X_MICROARCH.md
    'DVFS give-back');
  * held clock = those cycles / (End_Timestamp - Start_Timestamp);
  * MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x active cycles): the fraction of SIMD-cycles whose
    matrix pipe was busy, i.e. TFLOP/s relative to the peak at the clock the chip actually held.  (Checked on a
    4096^3 bf16 GEMM: this ratio equals TFLOP/s / (2.5 PF x held clock / 2.4 GHz) within a few percent.)
The 'all' line sums every matching dispatch, so it is the whole pass's time-weighted utilisation."""
import collections
import csv
import sqlite3
import sys

SIMDS = 256 * 4
XCDS = 8


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = "select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection"
        return [dict(zip(("Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp",
                          "End_Timestamp"), r)) for r in c.execute(q)]
    return list(csv.DictReader(open(path)))


def main():
    rows = load(sys.argv[1])
    pats = sys.argv[2:]
    disp = collections.defaultdict(dict)
    for r in rows:
        k = r["Kernel_Name"]
        if pats and not any(p in k for p in pats):
            continue
        d = disp[r["Dispatch_Id"]]
        d["name"] = k.split("(")[0].replace("void ", "")[-48:]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for d in disp.values():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
            continue
        for key in (d["name"], "all"):
            a = agg[key]
            a[0] += 1
            a[1] += d["ns"]
            a[2] += d["GRBM_GUI_ACTIVE"] / XCDS
            a[3] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
    print(f"{'kernel':50s} {'n':>5s} {'ms':>9s} {'GHz':>6s} {'mfma_util':>9s}")
    for k, (n, ns, cyc, busy) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:50s} {n:5d} {ns / 1e6:9.3f} {cyc / max(ns, 1):6.3f} {busy / max(SIMDS * cyc, 1):9.3f}")


if __name__ == "__main__":
    main()
