"""Static check of a built libwmx.so: no MFMA may execute under an EXEC mask that can be zero.

Root cause of the round-1 / round-2 packed-GEMM failures ("Guarded loads"): with per-step guarded
loads, LLVM (ROCm 7.2, gfx950) predicated some of the guarded MFMAs with `s_and_saveexec_b64` alone -- no
`s_cbranch_execz` around them -- treating EXEC = 0 as a no-op.  MFMA (MAI) instructions do not honour EXEC: they run
and accumulate whatever their operand registers hold, here the registers of the skipped loads (stale, NaN bit
patterns), so the outputs turned NaN (measured: gpurun_out r03a guarded_variant.log, NaN logits at step 0 with every
load address in bounds), and NaN logits made the top-K selection return its sentinel token id, which the next step's
embedding gather dereferenced: the illegal-address fault.

The check: extract the gfx950 code objects from the library's offload bundles, disassemble them with llvm-objdump,
and for every v_mfma walk back through its basic block: an EXEC-narrowing instruction (s_and_saveexec*, s_and*_b64
exec, ...) reached before a branch on EXEC (s_cbranch_execz / execnz) or a block boundary is a violation.
Usage: python tools/isa_exec_check.py <libwmx.so> [--verbose]   (exit 1 on violations)
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NARROW = re.compile(r"^s_(and|andn2|or|orn2|xor|mov|cselect)(_saveexec)?_b64\s+(exec|s\[\d+:\d+\]), ")
NARROW_SAVE = re.compile(r"^s_(and|andn2|or|orn2|xor)_saveexec_b64\s")


def code_objects(lib_path: str):
    """Every amdgcn code object of the library's offload bundles (bytes)."""
    data = open(lib_path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24: p + 24 + tlen].decode(errors="replace")
            p += 24 + tlen
            if "amdgcn" in triple and size:
                out.append((triple, data[pos + off: pos + off + size]))
        pos = data.find(MAGIC, pos + 24)
    return out


def disassemble(blob: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
        f.write(blob)
        path = f.name
    try:
        return subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", "--no-show-raw-insn", path], capture_output=True,
                              text=True, check=True).stdout
    finally:
        os.unlink(path)


def violations(asm: str):
    """(function, index, mfma line, narrowing line) for each MFMA whose block narrows EXEC without a branch on EXEC."""
    out = []
    func = None
    block = []  # instructions of the current basic block
    for raw in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", raw.strip())
        if m:
            func, block = m.group(1), []
            continue
        line = raw.strip()
        if not line or line.startswith(";") or func is None:
            continue
        ins = re.sub(r"\s*//.*$", "", line)
        ins = re.sub(r"^[0-9a-f]+:\s*", "", ins).strip()
        if not ins:
            continue
        if ins.startswith("v_mfma") or ins.startswith("v_smfmac"):
            for prev in reversed(block):
                if prev.startswith(("s_cbranch_execz", "s_cbranch_execnz")):
                    break  # a zero EXEC branches around
                if prev.startswith(("s_or_b64 exec, exec", "s_mov_b64 exec, -1", "s_mov_b64 exec, s")):
                    break  # EXEC restored (or set from a saved full mask) before the MFMA
                if NARROW_SAVE.match(prev) or (NARROW.match(prev) and prev.split()[1].startswith("exec")):
                    out.append((func, ins, prev))
                    break
        if ins.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
            block = []  # a branch ends the block; the fall-through starts a new one
        else:
            block.append(ins)
        # objdump marks branch targets as <label>: lines, handled above as a new function header only for symbols;
        # local targets appear as comments, so a conservative block split on every branch is what we can do
    return out


def main():
    lib = sys.argv[1]
    verbose = "--verbose" in sys.argv
    bad = []
    cos = code_objects(lib)
    if not cos:
        print("no amdgcn code objects found", file=sys.stderr)
        sys.exit(2)
    for triple, blob in cos:
        v = violations(disassemble(blob))
        bad += v
        if verbose:
            print(triple, len(blob), "bytes,", len(v), "violations")
    kern = sorted({f for f, _, _ in bad})
    print(f"{len(cos)} code objects, {len(bad)} MFMA(s) under a possibly-empty EXEC mask in {len(kern)} kernel(s)")
    for k in kern[:20]:
        print("  ", k)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
