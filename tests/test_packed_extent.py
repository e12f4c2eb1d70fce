"""Host-side bounds check of the decode GEMM (gemm_packed_kernel) for every launch shape the runtime emits.

A variant of this kernel that issued more fragments per load batch once faulted with an illegal address (DESIGN.md
§3, round 1).  The kept kernel shares its indexing, so every launch the runtime can make is walked here, on the CPU,
through the kernel's own index helpers (wmx_kernels.h packed_wave_ksteps / packed_w_elem / packed_a_elem via
wmx_debug_packed_launch) and compared with the allocation it addresses (wmx_runtime.hip build_model / alloc_ctx):
  * weights: a packed [N][K] tensor holds N x K elements (N multiple of 16); the token embedding ceil16(V) x d;
  * A operands: the context's decoder activations hold max(R, B x 448) rows x lda;
  * split-K partials: R x d x 48 floats.
No GPU is needed.
"""
import ctypes as C

import numpy as np
import pytest

from wmx import engine as E
from wmx._lib import check, lib

T_CTX = 448


def launch(M, N, K, part_cap, split, lda):
    out = np.zeros(9, np.int64)
    check(lib.wmx_debug_packed_launch(M, N, K, part_cap, split, lda, out.ctypes.data_as(C.POINTER(C.c_int64))))
    return dict(zip(("S", "MT", "NCT", "NW", "KU", "w_end", "a_end", "part_end", "stray"), map(int, out)))


def decode_launches(d, B, K):
    """(name, M, N, Kdim, split, lda, weight elements, A rows) of the packed launches of one decode step, the
    prefill / language / alignment passes that stay on the packed path (<= 256 rows) and the logits."""
    dt, V = d.n_text_state, d.n_vocab
    R = B * K
    rows_cap = max(R, B * T_CTX)
    logits_rows = max(R, 2 * B, 256)
    out = [("qkv", R, 3 * dt, dt, 1, dt, 3 * dt * dt, rows_cap),
           ("out", R, dt, dt, 1, dt, dt * dt, rows_cap),
           ("cross_q", R, dt, dt, 1, dt, dt * dt, rows_cap),
           ("fc1", R, 4 * dt, dt, 0, dt, 4 * dt * dt, rows_cap),
           ("fc2", R, dt, 4 * dt, 1, 4 * dt, 4 * dt * dt, rows_cap),
           ("logits", R, V, dt, 0, dt, (V + 15) // 16 * 16 * dt, rows_cap),
           # the LayerNorm-folded step (wmx_runtime.hip dec_step_fold): unsplit residual producers, 16 columns per
           # workgroup (split mode 2), and the folded QKV / cross-q / fc1 on the same shapes as above
           ("out_resid", R, dt, dt, 2, dt, dt * dt, rows_cap),
           ("fc2_resid", R, dt, 4 * dt, 2, 4 * dt, 4 * dt * dt, rows_cap)]
    # dec_forward on packed weights: rows x Tn <= 256 (more rows take the row-major tiled GEMM)
    for M in sorted({1, 2, 3, B, min(256, 3 * B), min(256, 7 * B), 255, 256}):
        if M > rows_cap:
            continue
        out += [("fwd_qkv", M, 3 * dt, dt, 0, dt, 3 * dt * dt, rows_cap),
                ("fwd_out", M, dt, dt, 0, dt, dt * dt, rows_cap),
                ("fwd_fc1", M, 4 * dt, dt, 0, dt, 4 * dt * dt, rows_cap),
                ("fwd_fc2", M, dt, 4 * dt, 0, 4 * dt, 4 * dt * dt, rows_cap)]
    for n in sorted({1, 2 * B, min(logits_rows, 64), logits_rows}):
        out.append(("logits_rows", n, V, dt, 0, dt, (V + 15) // 16 * 16 * dt, rows_cap))
    return out


CONTEXTS = [(B, K) for B in (1, 2, 3, 4, 5, 8, 16, 20) for K in (1, 5)]


@pytest.mark.parametrize("name", ["micro", "tiny", "base", "large-v3"])
def test_packed_launches_stay_inside_their_buffers(name):
    d = E.MODEL_DIMS[name]
    n = 0
    for B, K in CONTEXTS:
        R = B * K
        part_cap = R * d.n_text_state * 48
        for tag, M, N, Kd, split, lda, w_elems, a_rows in decode_launches(d, B, K):
            e = launch(M, N, Kd, part_cap, split, lda)
            where = (name, B, K, tag, M, N, Kd, e)
            assert e["stray"] == 0, where
            assert e["w_end"] <= w_elems, where
            assert e["a_end"] <= a_rows * lda, where
            assert (e["S"] == 1) == (split != 1), where
            if split == 2 and M <= 64:  # more rows: launch_packed_mt's 96- / 64-row configurations (NCT 2)
                assert e["NCT"] == 1, where
            if split:
                assert e["part_end"] <= part_cap, where
                assert e["S"] <= 8, where
            n += 1
    print(name, "packed launches checked:", n)


def test_extent_walker_is_tight():
    """The walker reports the exact end of what a launch reads: every weight element and every A row."""
    e = launch(20, 1280, 1280, 20 * 1280 * 48, 1, 1280)
    assert e["w_end"] == 1280 * 1280
    assert e["a_end"] == 19 * 1280 + 1280
    assert e["part_end"] == e["S"] * 20 * 1280
    assert (e["MT"], e["NCT"]) == (2, 2)
    f = launch(20, 1280, 5120, 20 * 1280 * 48, 1, 5120)
    assert f["NCT"] == 4 and f["w_end"] == 1280 * 5120
