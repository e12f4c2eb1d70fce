"""Kernel time of the stage that follows the decode loop (word alignment), per queue, from a rocprofv3
--kernel-trace CSV: for every queue, the kernels after the last decode-step kernel (`embed_ln_kernel`) of each
transcribe call up to the next `logmel_finalize_kernel`, summed by kernel name (tuning aid).

  python tools/stage_kernels.py <run_kernel_trace.csv>"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r.get("Queue_Id", r.get("Stream_Id"))].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-60:]))
    for q, ks in sorted(byq.items()):
        ks.sort()
        if len(ks) < 1000:
            continue
        # segments: after the last embed_ln before each logmel (and the final one)
        agg = collections.defaultdict(lambda: [0, 0])
        spans = 0
        i = 0
        n = len(ks)
        while i < n:
            # find next logmel or end
            j = i
            while j < n and "logmel_finalize" not in ks[j][2]:
                j += 1
            last = max((k for k in range(i, j) if "embed_ln" in ks[k][2]), default=None)
            if last is not None:
                spans += 1
                for s, e, name in ks[last + 1:j]:
                    agg[name][0] += 1
                    agg[name][1] += e - s
            i = j + 1
        tot = sum(v[1] for v in agg.values())
        print(f"queue {q}: {spans} post-decode spans, kernel time {tot / 1e6:.2f} ms ({tot / 1e6 / max(spans, 1):.2f} per span)")
        for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
            print(f"  {t / 1e6 / max(spans, 1):8.3f} ms/span n={c // max(spans, 1):5d} {name}")


if __name__ == "__main__":
    main()
