"""Memory-op / wait / barrier skeleton of one kernel in a hipcc --save-temps .s file: where the loads are issued,
what each s_waitcnt waits for, and whether readfirstlane waterfall loops wrap loads.
Usage: python tools/isa_audit.py <file.s> <mangled-name-substring> [--all]"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read()
    names = [n for n in re.findall(r"^(_Z\S+):", s, re.M) if pat in n]
    for nm in names[: (None if "--all" in sys.argv else 1)]:
        i = s.index(nm + ":")
        j = s.index(".Lfunc_end", i)
        body = [l.strip() for l in s[i:j].split("\n")]
        body = [l for l in body if l and not l.startswith(";") and not (l.startswith(".") and not l.startswith(".LBB"))]
        print(nm, "instructions:", len(body), "readfirstlane:", sum("v_readfirstlane" in l for l in body))
        keep = ("global_load", "global_store", "buffer_load", "buffer_store", "s_waitcnt", "s_barrier", "v_mfma",
                "ds_read", "ds_write", ".LBB", "s_cbranch", "s_endpgm", "global_atomic", "scratch_")
        out, last = [], None
        for l in body:
            if not l.startswith(keep):
                continue
            op = l.split()[0]
            if op == last and op.startswith(("v_mfma", "ds_read", "ds_write", "global_load", "buffer_load")):
                out[-1] = (out[-1][0], out[-1][1] + 1)
                continue
            out.append((l[:60] if op.startswith(("s_waitcnt", ".LBB", "s_cbranch")) else op, 1))
            last = op
        print("  " + " | ".join(f"{t} x{n}" if n > 1 else t for t, n in out))


if __name__ == "__main__":
    main()
