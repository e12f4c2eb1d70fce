"""Per-stream launch gaps from a rocprofv3 --kernel-trace CSV (tuning aid for the latency-bound decode loop).

  rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python bench.py --steps 1 --warmup 1 ...
  python tools/gap_stats.py <dir>/.../run_kernel_trace.csv [--min-ns N]

For every queue, kernels are sorted by start time; the gap before a kernel is its start minus the previous
kernel's end on the same queue (negative = overlap).  Prints, per next-kernel name, the count, the median and
mean duration and the median and mean gap, plus the share of the queue's span the kernels were busy."""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r[qkey]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-44:]))
    for q, ks in sorted(byq.items()):
        ks.sort()
        if len(ks) < 100:
            continue
        span = ks[-1][1] - ks[0][0]
        busy = sum(e - s for s, e, _ in ks)
        print(f"queue {q}: {len(ks)} kernels, span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({busy / span:.0%})")
        per = collections.defaultdict(lambda: ([], []))
        for (s0, e0, _), (s1, e1, n1) in zip(ks, ks[1:]):
            gap = s1 - e0
            if gap > 200000:  # host sync / chunk boundary: reported separately
                per["<gap > 200 us>"][1].append(gap)
                continue
            per[n1][0].append(e1 - s1)
            per[n1][1].append(gap)
        allg = [s1 - e0 for (s0, e0, _), (s1, e1, n1) in zip(ks, ks[1:]) if s1 - e0 <= 200000]
        for lo, hi in ((-10**9, 1000), (1000, 5000), (5000, 20000), (20000, 200001)):
            sel = [g for g in allg if lo <= g < hi]
            print(f"  gaps in [{max(lo, 0) / 1e3:.0f}, {hi / 1e3:.0f}) us: n={len(sel)} total {sum(sel) / 1e6:.2f} ms")
        for n, (d, g) in sorted(per.items(), key=lambda kv: -sum(kv[1][0]) - sum(kv[1][1])):
            dm = statistics.median(d) / 1e3 if d else 0.0
            print(f"  {n:46s} n={len(g):6d} dur med {dm:7.2f} us  gap med {statistics.median(g) / 1e3:7.2f} us"
                  f" mean {statistics.mean(g) / 1e3:7.2f} us  total gap {sum(g) / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
