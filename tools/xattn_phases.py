#!/usr/bin/env python3
"""Where the decode cross attention's time goes: the per-workgroup phase stamps of the probed layer
(WMX_PHASE_PROBE=1 WMX_PHASE_DUMP=<npz> python bench.py ...; wmx_ctx_probe_phases) of both context groups.

Prints, over every graph-replayed decode step: the launch's span (earliest start .. latest end over both groups), the
median / p90 of each phase of a workgroup (wave 0's clock at: start, query projection done, query tile ready, first
scores, P.V done, waves combined, ticket taken, end), the start skew, and the workgroup durations split by how many
workgroups shared the CU at the same time (HW_ID: se / sh / cu, XCC_ID)."""
import sys

import numpy as np

PH = ["proj", "qtile", "scores", "pv", "combine", "ticket", "merge/end"]


def main(path):
    z = np.load(path)
    khz = float(z["khz"])
    us = 1000.0 / khz
    groups = sorted(k for k in z.files if k.startswith("g"))
    rows = []  # (step, group, wg, stamps..., xcc, hw)
    for g in groups:
        a = z[g].astype(np.int64)
        for s in range(a.shape[0]):
            for wg in range(a.shape[1]):
                r = a[s, wg]
                if r[0] and r[7]:
                    rows.append((s, int(g[1:]), wg, *r))
    if not rows:
        print("no stamps")
        return
    R = np.array(rows, np.int64)
    st = R[:, 3:11]
    xcc, hw = R[:, 11], R[:, 12]
    cu_key = xcc * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
    steps = np.unique(R[:, 0])
    spans, skews, ends = [], [], []
    co = np.zeros(len(R), np.int64)
    for s in steps:
        m = R[:, 0] == s
        idx = np.nonzero(m)[0]
        t0, t1 = st[idx, 0].min(), st[idx, 7].max()
        spans.append((t1 - t0) * us)
        for g in np.unique(R[idx, 1]):
            mg = idx[R[idx, 1] == g]
            skews.append((st[mg, 0].max() - st[mg, 0].min()) * us)
        # workgroups overlapping in time on the same CU
        for i in idx:
            same = idx[(cu_key[idx] == cu_key[i]) & (st[idx, 0] < st[i, 7]) & (st[idx, 7] > st[i, 0])]
            co[i] = len(same)
        starts = st[idx, 0]
        ends.append(((st[idx, 7] - t0) * us))
    d = np.diff(st, axis=1) * us
    tot = (st[:, 7] - st[:, 0]) * us
    print(f"{len(steps)} steps, {len(R)} workgroup records, groups {groups}, tick {us * 1000:.1f} ns")
    print(f"launch span (both groups) median {np.median(spans):.2f} us, p90 {np.percentile(spans, 90):.2f}")
    print(f"start skew within a group median {np.median(skews):.2f} us, p90 {np.percentile(skews, 90):.2f}")
    print(f"workgroup duration median {np.median(tot):.2f} us, p90 {np.percentile(tot, 90):.2f}, max {tot.max():.2f}")
    for k, n in enumerate(PH):
        print(f"  {n:10s} median {np.median(d[:, k]):6.2f}  p90 {np.percentile(d[:, k], 90):6.2f}  "
              f"mean {d[:, k].mean():6.2f} us")
    for c in np.unique(co):
        m = co == c
        print(f"  co-resident workgroups on the CU {c}: {m.sum():6d} records, duration median "
              f"{np.median(tot[m]):.2f} us, p90 {np.percentile(tot[m], 90):.2f}; proj {np.median(d[m, 0]):.2f} "
              f"scores {np.median(d[m, 2]):.2f} pv {np.median(d[m, 3]):.2f}")
    # the last-arriving chunk (merge) vs the others
    mer = d[:, 6] > np.median(d[:, 6]) * 3
    print(f"  merging workgroups: {mer.sum()} (merge phase median {np.median(d[mer, 6]) if mer.any() else 0:.2f} us)")
    # start offset of each workgroup after the launch's first start, and its end
    off = []
    for s in steps:
        idx = np.nonzero(R[:, 0] == s)[0]
        off.extend((st[idx, 0] - st[idx, 0].min()) * us)
    print(f"  workgroup start offset from the launch's first start: median {np.median(off):.2f}, "
          f"p90 {np.percentile(off, 90):.2f}, max {np.max(off):.2f} us")
    print(f"  distinct CUs used per step: {np.mean([len(np.unique(cu_key[R[:, 0] == s])) for s in steps]):.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
