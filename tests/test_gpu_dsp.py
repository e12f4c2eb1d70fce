"""GPU parity of the pre-ASR DSP kernels (csrc/wmx_dsp.hip) against the reference modules' own outputs
(tests/golden/dsp_golden.npz): band-pass filtfilt within 1e-6 (fp64 recursion, fp32 output) and the dedup
feature vectors within 1e-5, all chunks of different lengths in one launch each."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "dsp_golden.npz"))
N = int(G["n"])


@pytest.fixture(scope="module")
def ctx():
    import torch
    torch.cuda.init()
    from wmx import engine
    m = engine.Model("micro", 0, "float16")
    m.init_synthetic(1)
    return engine.Context(m, max_batch=1, beam_size=1, max_new_tokens=8)


def test_filtfilt_batch_matches_reference(ctx):
    from wmx import dsp
    b, a = dsp.butter_bandpass(4, 85.0, 3400.0, 16000)
    xs = [G[f"x{i}"] for i in range(N)]
    ys = dsp.filtfilt_batch(ctx, xs, b, a)
    for i, y in enumerate(ys):
        err = float(np.max(np.abs(y - G[f"vocal{i}"])))
        assert err <= 1e-6, (i, len(xs[i]), err)


def test_separator_surface(ctx):
    from wmx import dsp
    sep = dsp.create_separator("filter", 16000, ctx=ctx, low_cut=85.0, high_cut=3400.0)
    vocal, bg = sep.separate(G["x0"])
    np.testing.assert_allclose(vocal, G["vocal0"], atol=1e-6)
    np.testing.assert_allclose(vocal + bg, G["x0"], atol=1e-6)
    short = np.ones(20, np.float32)
    v2, b2 = sep.separate(short)
    assert b2 is None and np.array_equal(v2, short)
    pairs = sep.separate_batch([G["x2"], short, G["x3"]])
    np.testing.assert_allclose(pairs[0][0], G["vocal2"], atol=1e-6)
    np.testing.assert_allclose(pairs[2][0], G["vocal3"], atol=1e-6)


def test_dedup_features_match_reference(ctx):
    from wmx import dsp
    xs = [G[f"x{i}"] for i in range(N)]
    f = dsp.dedup_features_batch(ctx, xs, 16000)
    np.testing.assert_allclose(f, G["feats"], rtol=1e-5, atol=1e-6)


def test_deduplicator_on_gpu_reproduces_reference_decisions(ctx):
    from wmx import dsp
    dd = dsp.AudioDeduplicator(ctx)
    got = []
    for i, t in zip(G["seq"], G["times"]):
        s, reason, _ = dd.should_skip(G[f"x{int(i)}"], 16000, current_time=float(t))
        got.append((int(s), {None: 0, "similar": 1, "duplicate": 2}[reason]))
    assert got == [tuple(r) for r in G["skips"]]


def test_mic_front_end_batches_streams_like_the_reference_loop(ctx):
    """3 streams x several chunk ticks: separation + dedup in one launch each per tick, per-stream decisions
    identical to running the oracle separator and deduplicator per stream (the reference loop order)."""
    from oracle import dsp_np as D
    from wmx import dsp
    sep = dsp.create_separator("filter", 16000, ctx=ctx)
    fe = dsp.MicFrontEnd(ctx, 3, separator=sep, dedup={"similarity_threshold": 0.95, "time_window": 3.0})
    refs = [dsp.AudioDeduplicator(features_fn=lambda a, sr: D.dedup_features(a, sr)) for _ in range(3)]
    order = [[0, 1, 0], [2, 2, 3], [4, 0, 0], [1, 1, 2]]  # golden chunk index per (tick, stream)
    for tick, ids in enumerate(order):
        t = 0.5 * tick
        xs = [G[f"x{j}"] for j in ids]
        got = fe.process(xs, current_time=t)
        for s_, j in enumerate(ids):
            v = D.filtfilt(sep.b, sep.a, G[f"x{j}"]).astype(np.float32)
            skip, _, _ = refs[s_].should_skip(v, 16000, current_time=t)
            assert (got[s_] is None) == skip, (tick, s_)
            if got[s_] is not None:
                np.testing.assert_allclose(got[s_], v, atol=1e-6)
