"""Wall-clock anatomy of the word-alignment stage from a rocprofv3 --kernel-trace CSV (tuning aid).

For every queue with a decode loop: the stage starts after the last decode-step kernel of a transcribe call (the
last `beam_update` / `greedy_update` before the call's alignment forward) and ends at the queue's last kernel before
the next call's `logmel` kernels. Reported per stage: the wall span, the summed kernel time, the idle gaps (the
largest ones named by the kernels around them), and kernel time by name.

  python tools/align_timeline.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

DECODE_END = ("beam_update", "greedy_update")
CALL_START = ("logmel",)


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r.get("Queue_Id", r.get("Stream_Id"))].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-70:]))
    for q, ks in sorted(byq.items()):
        ks.sort()
        if len(ks) < 1000:
            continue
        # the alignment forward is the first run of cross_scores kernels after a decode loop: walk back from each
        # cross_scores cluster to the last decode-end kernel, forward to the next logmel (or the queue's end)
        idx = [i for i, k in enumerate(ks) if "cross_scores" in k[2]]
        if not idx:
            continue
        clusters = [idx[0]]
        for a, b in zip(idx, idx[1:]):
            if b - a > 2000:
                clusters.append(b)
        for ci, c0 in enumerate(clusters, 1):
            s = c0
            while s > 0 and not any(t in ks[s - 1][2] for t in DECODE_END):
                s -= 1
            e = c0
            while e + 1 < len(ks) and not any(t in ks[e + 1][2] for t in CALL_START):
                e += 1
            seg = ks[s:e + 1]
            wall = seg[-1][1] - seg[0][0]
            busy = sum(x[1] - x[0] for x in seg)
            gaps = []
            for a, b in zip(seg, seg[1:]):
                g = b[0] - a[1]
                if g > 0:
                    gaps.append((g, a[2], b[2]))
            gaps.sort(reverse=True)
            agg = collections.defaultdict(lambda: [0, 0])
            for x in seg:
                agg[x[2]][0] += 1
                agg[x[2]][1] += x[1] - x[0]
            print(f"queue {q} stage {ci}: {len(seg)} kernels, wall {wall / 1e6:.2f} ms, kernel time {busy / 1e6:.2f} ms, "
                  f"idle {sum(g[0] for g in gaps) / 1e6:.2f} ms in {len(gaps)} gaps")
            for g, a, b in gaps[:8]:
                print(f"    gap {g / 1e3:8.1f} us after {a[-40:]} before {b[-40:]}")
            for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:16]:
                print(f"    {t / 1e3:9.1f} us n={n:5d} {name}")


if __name__ == "__main__":
    main()
