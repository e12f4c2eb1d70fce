"""GPU parity of the MX-fp8 encoder (model compute_type "float8", BASELINE config 5): the four projections of every
encoder layer on v_mfma_scale_f32_16x16x128_f8f6f4 with MX-fp8 activations produced by the LayerNorm, the
attention epilogue and the fc1 GELU epilogue.

Oracle: oracle/whisper_np.py encoder(..., mx8=True) on the same bf16-rounded weights (both operands of each
projection quantized with the same OCP MX rule, fp32 accumulation).  Tolerance: relative L2 <= 3e-2 (the bf16
path's bound: q/k/v and the attention stay bf16, and an activation whose f32 value differs in the last bits
from the oracle's may round to the neighbouring e4m3 code).  The fp8 model's distance to the bf16 model is
printed for reference.  Translate task: every greedy step whose oracle margin exceeds 0.15 equals the oracle's
argmax on the device's own path (>= 4 per window)."""
import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

pytestmark = pytest.mark.gpu

WIDE = O.Dims(128, 51866, 1280, 20, 2, 1280, 20, 1)


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _dims(E, d):
    return E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                       d.n_text_head, d.n_text_layer)


@pytest.mark.parametrize("name", ["micro", "wide"])
def test_mx8_encoder_matches_oracle(name):
    from wmx import engine as E
    d = O.DIMS["micro"] if name == "micro" else WIDE
    m = E.Model(_dims(E, d), 0, "float8").init_synthetic(9)
    ctx = E.Context(m, max_batch=3, beam_size=1, max_new_tokens=8, word_timestamps=False)
    W = O.make_weights(d, 9, "bf16")
    mels = np.stack([O.logmel_segment(synth.speech_like(s, n), d.n_mels)
                     for s, n in ((81, 480000), (82, 200000), (83, 60000))])
    got = ctx.encode(mels)
    for b in range(3):
        ref = O.encoder(W, d, mels[b], mx8=True)
        e = rel_l2(got[b], ref)
        e16 = rel_l2(got[b], O.encoder(W, d, mels[b]))
        print(name, "mx8 encoder window", b, "rel_l2 vs mx8 oracle", e, "| vs bf16 oracle", e16)
        assert e <= 3e-2, (b, e)


def test_mx8_translate_greedy_matches_oracle():
    from wmx import engine as E
    d = O.DIMS["micro"]
    m = E.Model("micro", 0, "float8").init_synthetic(9)
    ctx = E.Context(m, max_batch=2, beam_size=1, max_new_tokens=24, task="translate", word_timestamps=False)
    W = O.make_weights(d, 9, "bf16")
    audios = [synth.speech_like(91, 480000), synth.speech_like(92, 96000)]
    res = ctx.transcribe(audios)
    from test_gpu_parity import greedy_forced_compare
    per = []
    for a, r in zip(audios, res):
        enc = O.encoder(W, d, O.logmel_segment(a, d.n_mels), mx8=True)
        lang, _ = O.detect_language(W, d, enc)
        assert r.language == lang
        opt = O.DecodeOptions(language=lang, beam_size=1, max_new_tokens=24, task="translate")
        n, _ = greedy_forced_compare(W, d, enc, opt, r.tokens, 0.15)
        per.append(n)
    print("mx8 translate greedy steps compared per window", per)
    assert min(per) >= 4, per


def test_mx8_full_depth_large_v3_translate():
    """Config 5's model at full depth: large-v3 with the MX-fp8 encoder (32 layers), window 0 of three, against the
    oracle's MX rule, then the translate task's first greedy steps replayed token-exact on the recorded logits."""
    from wmx import engine as E
    import test_gpu_step as S
    d = O.DIMS["large-v3"]
    sp = O.special_tokens(d.n_vocab)
    m = E.Model("large-v3", 0, "float8").init_synthetic(1)
    W = {name: m.get_tensor(name, shape) for name, shape, _, _ in O.tensor_specs(d)}
    W["encoder.embed_positions.weight"] = O.sinusoids(1500, d.n_audio_state)
    audio = synth.speech_like(511, 480000)
    mel = O.logmel_segment(audio, d.n_mels)
    # three windows (4500 rows): the encoder projections run on the 256 x 256 / 32x32x64 MX-fp8 GEMM (from 4096
    # rows); window 0 is compared
    mels = np.stack([mel] + [O.logmel_segment(synth.speech_like(s, 240000), d.n_mels) for s in (512, 513)])
    ctx = E.Context(m, max_batch=3, beam_size=1, max_new_tokens=8, task="translate", word_timestamps=False)
    got = ctx.encode(mels)[0]
    ref = O.encoder(W, d, mel, mx8=True)
    e = rel_l2(got, ref)
    e16 = rel_l2(got, O.encoder(W, d, mel))
    print("large-v3 full-depth MX-fp8 encoder rel_l2", e, "| vs bf16 oracle", e16)
    # 32 layers compound the e4m3 rounding-boundary flips (an f32 value a few ulps from the oracle's rounds to the
    # neighbouring code, one e4m3 step = 6-12 %): measured 3.3e-2 here against 0.9-1.1e-2 at 2 layers; the bound
    # is 5e-2, and the device must sit at most half as far from the MX-fp8 oracle as the MX-fp8 model sits from
    # the bf16 one (7.3e-2 measured)
    assert e <= 5e-2, e
    assert e <= 0.5 * e16, (e, e16)
    ctx.record(8)
    res = ctx.transcribe([audio])
    opt = O.DecodeOptions(beam_size=1, max_new_tokens=8, task="translate")
    S._replay_and_compare("large-v3 full depth MX-fp8 translate greedy", ctx, res, 1, opt, sp, 1)
