"""Per-kernel-kind PMC summary of an encoder pass (tools/encprof.py under rocprofv3 --pmc, CSV output).

  pass 1: --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE       -> held clock, MFMA-pipe busy fraction of SIMD-cycles
  pass 2: --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
                                                               -> where the waves' cycles go (MI355X_MICROARCH.md PMC table)
Usage: python tools/enc_pmc.py <pass-1 counter_collection.csv> [<pass-2 counter_collection.csv>]"""
import collections
import csv
import sys

SIMDS, XCDS = 256 * 4, 8


def per_kind(path):
    disp = collections.defaultdict(dict)
    with open(path) as f:
        for r in csv.DictReader(f):
            d = disp[r["Dispatch_Id"]]
            nm = r["Kernel_Name"].replace("void ", "").replace("wmx::", "").replace("(DT)", "")
            d["name"] = nm[:nm.find(">(") + 1] if ">(" in nm else nm.split("(")[0]
            d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in disp.values():
        a = agg[d["name"]]
        a["n"] += 1
        for k, v in d.items():
            if k != "name":
                a[k] += v
    return agg


p1 = per_kind(sys.argv[1])
p2 = per_kind(sys.argv[2]) if len(sys.argv) > 2 else {}
print(f"{'kernel':34s} {'n':>4s} {'us/launch':>9s} {'GHz':>6s} {'mfma':>6s} | {'wait':>6s} {'stall':>6s} {'issue':>6s} {'lds':>6s}")
tot = collections.defaultdict(float)
for k, a in sorted(p1.items(), key=lambda kv: -kv[1]["ns"]):
    if a["ns"] < 1e5:
        continue
    cyc = a["GRBM_GUI_ACTIVE"] / XCDS
    line = f"{k[:34]:34s} {int(a['n']):4d} {a['ns'] / a['n'] / 1e3:9.1f} {cyc / a['ns']:6.3f} " \
           f"{a['SQ_VALU_MFMA_BUSY_CYCLES'] / max(SIMDS * cyc, 1):6.3f}"
    for key in ("ns", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"):
        tot[key] += a[key]
    b = p2.get(k)
    if b and b.get("SQ_WAVE_CYCLES"):
        w = b["SQ_WAVE_CYCLES"]
        line += f" | {b['SQ_WAIT_ANY'] / w:6.3f} {b['SQ_WAIT_INST_ANY'] / w:6.3f} {b['SQ_ACTIVE_INST_ANY'] / w:6.3f} " \
                f"{b.get('SQ_WAIT_INST_LDS', 0) / w:6.3f}"
    print(line)
cyc = tot["GRBM_GUI_ACTIVE"] / XCDS
print(f"{'all (listed)':34s} {'':4s} {tot['ns'] / 1e3:9.1f} {cyc / max(tot['ns'], 1):6.3f} "
      f"{tot['SQ_VALU_MFMA_BUSY_CYCLES'] / max(SIMDS * cyc, 1):6.3f}   (total us)")
