"""The root cause of the packed-GEMM faults of rounds 1-2 ("Guarded loads"), as a CPU-side check of
the built library: no MFMA may execute under an EXEC mask that can be zero.

LLVM (ROCm 7.2, gfx950) may predicate a divergent-looking `if` around MFMAs with `s_and_saveexec` alone, treating
EXEC = 0 as a no-op; MFMA instructions ignore EXEC and accumulate whatever their operand registers hold.  With
per-step guarded loads those registers were stale (NaN bit patterns): the guarded variant produced NaN logits at the
first step with every load address in bounds (profiles/r03a_guarded_variant.log; its bounds-checked build reported
no out-of-range load).  tools/isa_exec_check.py disassembles the library's gfx950 code objects and flags every such
MFMA; it must find none in the shipped libwmx.so, and it must find the guarded variant's (the check has teeth) when
that diagnostic build is present."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "realtime-whisper-asr_amd", "wmx", "libwmx.so")
GUARDED = os.path.join(ROOT, "realtime-whisper-asr_amd", "wmx", "libwmx_guarded.so")
CHECK = os.path.join(ROOT, "tools", "isa_exec_check.py")


def _run(lib):
    return subprocess.run([sys.executable, CHECK, lib], capture_output=True, text=True, timeout=300)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libwmx.so not built")
def test_no_mfma_under_possibly_empty_exec():
    r = _run(LIB)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 MFMA(s)" in r.stdout


@pytest.mark.skipif(not os.path.exists(GUARDED), reason="diagnostic build (tools/build_variant.sh guarded "
                                                         "-DWMX_PACKED_GUARDED) not present")
def test_check_flags_the_guarded_variant():
    r = _run(GUARDED)
    assert r.returncode == 1 and "gemm_packed_kernel" in r.stdout, r.stdout
