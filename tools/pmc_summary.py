"""Average rocprofv3 --pmc counters per (kernel, grid) from a run_counter_collection.csv (tuning aid).
Usage: python tools/pmc_summary.py <run_counter_collection.csv> [kernel-substring ...]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    pats = sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"]
        if pats and not any(p in k for p in pats):
            continue
        agg[(k.split("(")[0][-40:], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (k, g), d in sorted(agg.items()):
        m = {c: sum(v) / len(v) for c, v in d.items()}
        print(k, "grid", g, " ".join(f"{c}={m[c]:.3g}" for c in sorted(m)))


if __name__ == "__main__":
    main()
