"""GPU parity at large-v3 WIDTH: d = 1280, 20 heads, 128 mels, vocab 51866, one encoder and one decoder layer.

The micro model (d = 128) never reaches the large-v3-only code paths; this one does, on three windows at once:
  * the 256 x 256 encoder GEMM tile with every epilogue kind (GELU, fp32 residual, conv2 GELU + position, and the
    head-major fragment-major cross-K/V scatter, which needs d % 256 == 0),
  * the 32x32x16 encoder self-attention with 20 heads,
  * the decode cross attention over 20 heads, key-chunked (5 queries per window) and whole (21 queries).
Tolerances as tests/test_gpu_parity.py: relative L2 vs the fp32 oracle on dtype-rounded weights, bf16 <= 3e-2,
f16 <= 5e-3.
"""
import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

pytestmark = pytest.mark.gpu

WIDE = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 1)
REL = {"bf16": 3e-2, "f16": 5e-3}
DT = {"bf16": "bfloat16", "f16": "float16"}


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module", params=["bf16", "f16"])
def wide(request):
    from wmx import engine as E
    dt = request.param
    dims = E.ModelDims(WIDE.n_mels, WIDE.n_vocab, WIDE.n_audio_state, WIDE.n_audio_head, WIDE.n_audio_layer,
                       WIDE.n_text_state, WIDE.n_text_head, WIDE.n_text_layer)
    m = E.Model(dims, 0, DT[dt]).init_synthetic(5)
    ctx = E.Context(m, max_batch=3, beam_size=1, max_new_tokens=8, word_timestamps=False)
    W = O.make_weights(WIDE, 5, dt)
    mels = np.stack([O.logmel_segment(synth.speech_like(s, n), 128)
                     for s, n in ((71, 480000), (72, 150000), (73, 320000))])
    encs = [O.encoder(W, WIDE, mel) for mel in mels]
    return dt, m, ctx, W, mels, encs


def test_wide_encoder_matches_oracle(wide):
    dt, _, ctx, _, mels, encs = wide
    got = ctx.encode(mels)
    for b in range(3):
        e = rel_l2(got[b], encs[b])
        print(dt, "wide encoder window", b, "rel_l2", e)
        assert e <= REL[dt], (b, e)


def test_wide_decoder_logits_match_oracle(wide):
    dt, _, ctx, W, mels, encs = wide
    sp = O.special_tokens(WIDE.n_vocab)
    ctx.encode(mels, want_output=False)
    rng = np.random.default_rng(11)
    for T in (5, 21):
        toks = np.concatenate([np.full((3, 1), sp.sot, np.int32),
                               rng.integers(0, 50000, size=(3, T - 1)).astype(np.int32)], axis=1)
        got = ctx.decoder_logits(toks)
        for b in range(3):
            ref = O.decoder_forward(W, WIDE, list(toks[b]), O.DecoderCache(W, WIDE, encs[b]))
            e = rel_l2(got[b], ref)
            print(dt, "wide T", T, "window", b, "rel_l2", e)
            assert e <= REL[dt], (T, b, e)
