"""Static check of a built libwmx.so: which kernels use scratch (a private segment, i.e. spilled or stack-allocated
registers), from the AMDGPU metadata notes of the library's gfx950 code objects.

Why: a few-microsecond decode launch that touches scratch pays a memory round trip per spilled value, and the
compiler demotes a whole struct to scratch when any member is reached through a selected pointer (round 4: the
folded-LayerNorm prefetch struct put 80-448 bytes of scratch into every S == 1 packed-GEMM instantiation, and the
mixed step's fc1 went from 10.6 to 15.9 us in situ).  tests/test_isa_exec.py asserts that none of the decode-step and
encoder kernels below carries a private segment.
Usage: python tools/scratch_check.py <libwmx.so> [--all]   (prints name, private segment bytes, VGPR spills)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_exec_check import code_objects  # noqa: E402

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def kernels(lib_path: str):
    """{kernel symbol: (private_segment_fixed_size, vgpr_spill_count)} over every gfx950 code object."""
    out = {}
    for _triple, blob in code_objects(lib_path):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(blob)
            path = f.name
        try:
            notes = subprocess.run([READELF, "--notes", path], capture_output=True, text=True, check=True).stdout
        finally:
            os.unlink(path)
        for block in notes.split("\n  - ")[1:]:
            name = re.search(r"^\s*\.name:\s+(\S+)$", block, re.M)
            priv = re.search(r"^\s*\.private_segment_fixed_size:\s+(\d+)$", block, re.M)
            spill = re.search(r"^\s*\.vgpr_spill_count:\s+(\d+)$", block, re.M)
            if name and priv:
                out[name.group(1)] = (int(priv.group(1)), int(spill.group(1)) if spill else 0)
    return out


def main():
    ks = kernels(sys.argv[1])
    show_all = "--all" in sys.argv
    n = 0
    for name, (priv, spill) in sorted(ks.items()):
        if priv or spill or show_all:
            print(f"{priv:6d} {spill:4d}  {name}")
            n += priv > 0
    print(f"{n} of {len(ks)} kernels use scratch")


if __name__ == "__main__":
    main()
