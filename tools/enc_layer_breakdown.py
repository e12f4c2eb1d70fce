"""Per-launch durations of one encoder layer from a rocprofv3 --kernel-trace of tools/encprof.py (last pass, layers
2..31 averaged by position).  Usage: python tools/enc_layer_breakdown.py <run_kernel_trace.csv | rocpd .db>"""
import csv
import sqlite3
import sys

src = sys.argv[1]
if src.endswith(".csv"):
    with open(src) as f:
        rd = csv.DictReader(f)
        rows = sorted(((int(r["Start_Timestamp"]), r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
                       for r in rd))
    rows = [(n, d) for _, n, d in rows]
else:
    c = sqlite3.connect(src)
    rows = c.execute("select k.name, k.duration from kernels k order by k.start").fetchall()
rows = [(n.split("(")[0].replace("void ", "").replace("wmx::", ""), d / 1000) for n, d in rows if "rocclr" not in n]
first = max(i for i, r in enumerate(rows) if r[0].startswith("im2col1"))  # the last encoder pass
last = rows[first:]
last = last[:max(i for i, r in enumerate(last) if r[0].startswith("layernorm")) + 1]
# a layer starts at the launch two before the attention (a layernorm, or the folded producer's successor)
att = [i for i, r in enumerate(last) if "attn" in r[0]]
starts = [a - 2 for a in att]
layers = [last[a:b] for a, b in zip(starts, starts[1:])]
L = len(layers[0])
avg = [sum(l[j][1] for l in layers[1:]) / len(layers[1:]) for j in range(L)]
for j in range(L):
    print(f"{layers[0][j][0][:44]:46s} {avg[j]:8.1f} us")
print(f"layer total {sum(avg):.1f} us, {len(layers) + 1} layers, pass {sum(d for _, d in last) / 1000:.2f} ms")
