"""The library's own word-alignment DTW (wmx_runtime.hip dtw(), the path wmx_transcribe runs on the host after the
alignment-head kernels) on the committed DTW golden vectors (tests/golden/golden.npz dtw/*: HF
`_dynamic_time_warping`, the same fixtures that pin oracle.dtw in test_oracle_golden.py).  Host-only entry point
wmx_debug_dtw: no GPU needed."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "realtime-whisper-asr_amd"))


@pytest.fixture(scope="module")
def lib():
    from wmx import _lib
    return _lib.lib


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"))


def _dtw(lib, cost):
    x = np.ascontiguousarray(-np.asarray(cost, np.float32))  # the library takes the alignment matrix (cost = -x)
    N, M = x.shape
    ti = np.zeros(N + M, np.int32)
    tj = np.zeros(N + M, np.int32)
    n = C.c_int(0)
    st = lib.wmx_debug_dtw(x.ctypes.data_as(C.POINTER(C.c_float)), N, M, M, ti.ctypes.data_as(C.POINTER(C.c_int32)),
                           tj.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(n))
    assert st == 0, lib.wmx_last_error()
    return ti[: n.value], tj[: n.value]


def test_library_dtw_matches_golden(lib, golden):
    keys = sorted({k.split("/")[1] for k in golden.files if k.startswith("dtw/")})
    assert keys
    for i in keys:
        ti, tj = _dtw(lib, golden[f"dtw/{i}/x"])
        np.testing.assert_array_equal(ti, golden[f"dtw/{i}/ti"])
        np.testing.assert_array_equal(tj, golden[f"dtw/{i}/tj"])


def test_library_dtw_matches_oracle_on_ties_and_shapes(lib):
    import oracle.whisper_np as O
    rng = np.random.default_rng(7)
    for N, M in [(1, 1), (1, 9), (9, 1), (7, 31), (40, 300)]:
        for quant in (None, 0.25):  # quantised costs: many exact ties, the tie-breaking order matters
            cost = rng.standard_normal((N, M)).astype(np.float32)
            if quant:
                cost = (np.round(cost / quant) * quant).astype(np.float32)
            ti, tj = _dtw(lib, cost)
            oi, oj = O.dtw(cost)
            np.testing.assert_array_equal(ti, oi)
            np.testing.assert_array_equal(tj, oj)
