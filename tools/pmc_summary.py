"""Averages rocprofv3 counter_collection.csv rows per (kernel, counter) for kernels matching a pattern:
python tools/pmc_summary.py <dir> <kernel substring>"""
import collections
import csv
import glob
import os
import sys

root, pat = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if pat in name:
                acc[(name[:60], row["Counter_Name"])].append(float(row["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:60s} {c:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
