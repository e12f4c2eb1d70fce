"""The root cause of the packed-GEMM faults of rounds 1-2 ("Guarded loads"), as a CPU-side check of
the built library: no MFMA may execute under an EXEC mask that can be zero.

LLVM (ROCm 7.2, gfx950) may predicate a divergent-looking `if` around MFMAs with `s_and_saveexec` alone, treating
EXEC = 0 as a no-op; MFMA instructions ignore EXEC and accumulate whatever their operand registers hold.  With
per-step guarded loads those registers were stale (NaN bit patterns): the guarded variant produced NaN logits at the
first step with every load address in bounds (profiles/r03a_guarded_variant.log; its bounds-checked build reported
no out-of-range load).  tools/isa_exec_check.py disassembles the library's gfx950 code objects and flags every such
MFMA; it must find none in the shipped libwmx.so (round 3 checked that it flags the guarded variant's; that
diagnostic build was removed in round 6)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "realtime-whisper-asr_amd", "wmx", "libwmx.so")
CHECK = os.path.join(ROOT, "tools", "isa_exec_check.py")


def _run(lib):
    return subprocess.run([sys.executable, CHECK, lib], capture_output=True, text=True, timeout=300)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libwmx.so not built")
def test_no_mfma_under_possibly_empty_exec():
    r = _run(LIB)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 MFMA(s)" in r.stdout


# Kernels allowed a private segment (tools/scratch_check.py), each for a stated reason; any other kernel that grows
# one fails here, so a register-pressure regression on the decode / encoder path is caught at build time (round 4:
# a prefetch struct demoted to scratch in every S == 1 packed-GEMM instantiation cost the mixed step's fc1 5 us).
SCRATCH_ALLOWED = [
    (r"gemm256_kernelILNS_2DTE\dELin1E", "generic-epilogue fallback for N % 4 != 0 (no hot-path shape)"),
    (r"gemm256_kernelILNS_2DTE1ELi11E", "f16 only, 12 bytes"),
    (r"gemm_mx8_256_kernelILNS_2DTE\dELi2E", "MX-fp8 residual epilogue, 3 dwords outside the main loop"),
    (r"gemm_mx8_256_kernelILNS_2DTE\dELi7E",
     "MX-fp8 GELU->MX8 on the 128-deep ring: 6 dwords saved at entry, reloaded outside the steady-state K loop"),
    (r"enc_attn_kernelILNS_2DTE\dELi8ELi4E", "one VGPR stored before and reloaded after the key loop"),
    (r"dec_cross_attn_kernelILNS_2DTE\dELi[12]ELi\dELb\dELb0E",
     "16-bit images at <= 2 key blocks per wave under the 128-VGPR cap (not the default 1024-key decode chunk)"),
]


@pytest.mark.skipif(not os.path.exists(LIB), reason="libwmx.so not built")
def test_no_unexpected_scratch():
    import re

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from scratch_check import kernels

    ks = kernels(LIB)
    assert len(ks) > 100
    bad = [n for n, (priv, _spill) in ks.items() if priv and not any(re.search(p, n) for p, _ in SCRATCH_ALLOWED)]
    assert not bad, "kernels with an unexpected private segment:\n" + "\n".join(bad)
    # the default decode kernels are in the library and scratch-free
    for pat in (r"dec_cross_attn_kernelILNS_2DTE0ELi4ELi8ELb1ELb0ELb0E", r"dec_cross_attn_kernelILNS_2DTE0ELi2ELi8ELb1ELb1ELb0E",
                r"gemm_packed_kernelILNS_2DTE0ELi2ELi4ELi16ELi2ELi0E", r"dec_self_attn_kernel",
                # the int8 model's decode (f16 activations, int8 weights: split-K partials and the GELU fc1)
                r"gemm_packed_kernelILNS_2DTE1ELi2ELi2ELi8ELi0ELi2E", r"gemm_packed_kernelILNS_2DTE1ELi2ELi2ELi16ELi1ELi2E"):
        hits = [n for n in ks if re.search(pat, n)]
        assert hits and all(ks[n][0] == 0 for n in hits), pat


@pytest.mark.skipif(not os.path.exists(LIB), reason="libwmx.so not built")
def test_logmel_has_no_packed_f32_valu():
    """The log-mel front end is built without SLP-packed f32 arithmetic (Makefile: wmx_logmel.o with
    -fno-slp-vectorize).  With v_pk_fma/add/mul_f32 in it, its FFT kernel returned wrong frames while sharing CUs with
    another context's MFMA GEMM waves (4-17 of 15 concurrent calls, tools/conc_probe4.py); without them, 0 of 60
    (DESIGN.md 0e).  A build that loses the flag fails here, on the CPU."""
    import re

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from isa_exec_check import code_objects, disassemble

    seen, packed = set(), []
    for _triple, blob in code_objects(LIB):
        func = None
        for raw in disassemble(blob).splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", raw.strip())
            if m:
                func = m.group(1) if "logmel" in m.group(1) else None
                if func:
                    seen.add(func)
                continue
            if func and re.search(r"\bv_pk_(fma|add|mul)_f32\b", raw):
                packed.append((func, raw.strip()))
    assert any("logmel_fft_kernel" in f for f in seen), sorted(seen)
    assert not packed, packed[:5]
