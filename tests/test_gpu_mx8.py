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
    W = O.fp8_decoder_weights(O.make_weights(d, 9, "bf16"), d)  # (the MX-fp8 encoder + the fp8 decode)
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


# ---------------------------------------------------------------------------------------------------------------
# the fp8 decode (round 4): every decoder projection and the logits projection on 8-bit weights (e4m3, one
# power-of-two scale per weight row, widened to bf16 in registers, the row scale on the fp32 result) and the cross
# K / V images in e4m3 (one power-of-two scale per (layer, window, head) image).  Oracle: oracle.fp8_decoder_weights
# (the same rules in numpy: w8_rows, kv8_images) on the DEVICE's own encoder output, so the comparison isolates the
# decoder.  Tolerance: the bf16 step bound, relative L2 <= 3e-2 per row and step, and argmax equality wherever the
# oracle's top-2 margin exceeds twice the row's max abs error (tests/test_gpu_step.py _check_forced); both sides use
# bit-identical dequantized weights, so what is left is bf16 activation rounding and the image element rounding of
# the device's 16-bit K / V (the oracle rounds its fp32 K / V to bf16 first, as the device stores them).
# ---------------------------------------------------------------------------------------------------------------
WIDE2 = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 2)  # large-v3 width, 1 encoder layer, 2 decoder layers


@pytest.fixture(scope="module")
def wide_fp8():
    from wmx import engine as E
    m = E.Model(_dims(E, WIDE2), 0, "float8").init_synthetic(5)
    W = O.fp8_decoder_weights(O.make_weights(WIDE2, 5, "bf16"), WIDE2)
    lens = [480000, 150000, 320000, 16000, 240000, 480000, 90000, 400000]
    mels = np.stack([O.logmel_segment(synth.speech_like(300 + i, n), 128) for i, n in enumerate(lens)])
    return m, W, mels


@pytest.mark.parametrize("B,K", [(4, 5), (8, 5), (20, 1)])
def test_fp8_decode_forced_steps_wide(wide_fp8, B, K):
    """Teacher-forced decode steps of the fp8 decode at large-v3 width: 4 and 8 windows x beam 5 (R = 20 and 40, the
    bench's per-group rows at 8 and 16 windows per GPU) and 20 windows greedy, 24 steps, parents re-drawn every
    step."""
    from wmx import engine as E
    import test_gpu_step as S
    m, W, mels = wide_fp8
    sp = O.special_tokens(WIDE2.n_vocab)
    ctx = E.Context(m, max_batch=B, beam_size=K, max_new_tokens=64, word_timestamps=False)
    mel = np.concatenate([mels] * 3)[:B]
    encs = list(ctx.encode(mel))
    n = 24
    tok, par = S._forced_stream(np.random.default_rng(7 + B), n, B * K, K)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]] * B
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, WIDE2, encs, prefix, tok, par, K)
    S._check_forced(f"fp8 decode B={B} K={K}", "bf16", top1, lg, 1, ref_top1, ref_margin, ref_lg, 16)
    # the fp8 model sits measurably away from the bf16 one (the quantization is live, not a no-op)
    W16 = O.make_weights(WIDE2, 5, "bf16")
    _, _, lg16 = O.forced_rows(W16, WIDE2, encs[:1], prefix[:1], tok[:2, :K], par[:2, :K], K)
    d16 = rel_l2(lg[1, 0], lg16[1][0])
    print("fp8 decode vs bf16 decode weights, row 0 step 1 rel_l2", d16)
    assert d16 > 5e-3, d16


def test_fp8_decode_search_replay_wide(wide_fp8):
    """Free-running beam-5 transcribe of 8 windows (config 5's per-group shape at 16 windows per GPU), translate,
    recorded: the oracle replays the rules / beam bookkeeping on the device's logits and must choose exactly the
    device's selection at every step, and rank the device's final sequence."""
    from wmx import engine as E
    import test_gpu_step as S
    m, W, mels = wide_fp8
    sp = O.special_tokens(WIDE2.n_vocab)
    audios = [synth.speech_like(300 + i, n) for i, n in
              enumerate([480000, 150000, 320000, 16000, 240000, 480000, 90000, 400000])]
    ctx = E.Context(m, max_batch=8, beam_size=5, max_new_tokens=32, task="translate", word_timestamps=True,
                    language=sp.lang0)
    ctx.record(33)
    res = ctx.transcribe(audios)
    opt = O.DecodeOptions(language=sp.lang0, beam_size=5, max_new_tokens=32, task="translate")
    S._replay_and_compare("fp8 decode beam5 B=8 translate", ctx, res, 5, opt, sp, 16)
    assert all(r.jump_times is not None for r in res)


def test_fp8_decode_full_depth_large_v3():
    """Config 5's model at full depth (32 + 32 layers, vocab 51866): 8 teacher-forced steps of one window x beam 5
    against the fp8 oracle on the device's encoder output."""
    from wmx import engine as E
    import test_gpu_step as S
    d = O.DIMS["large-v3"]
    sp = O.special_tokens(d.n_vocab)
    m = E.Model("large-v3", 0, "float8").init_synthetic(1)
    W = {name: m.get_tensor(name, shape) for name, shape, _, _ in O.tensor_specs(d)}
    W["encoder.embed_positions.weight"] = O.sinusoids(1500, d.n_audio_state)
    W = O.fp8_decoder_weights(W, d)
    ctx = E.Context(m, max_batch=1, beam_size=5, max_new_tokens=16, word_timestamps=False)
    encs = list(ctx.encode(O.logmel_segment(synth.speech_like(611, 480000), d.n_mels)[None]))
    n = 8
    tok, par = S._forced_stream(np.random.default_rng(11), n, 5, 5)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]]
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, d, encs, prefix, tok, par, 5)
    S._check_forced("fp8 decode large-v3 full depth", "bf16", top1, lg, 1, ref_top1, ref_margin, ref_lg, 4)


def _alignment_legs(ct):
    """The word-alignment pass of one model (compute type ct) on two windows at large-v3 width with the large-v3
    alignment heads, against oracle.find_alignment on the same weights (fp8: the fp8 decoder rule) and the device's own
    encoder output.  Returns per window (matrix rel-L2, fraction of jump times within one frame, tokens off by more
    than one frame, text tokens)."""
    from wmx import engine as E
    import test_gpu_align as A
    d = A.ALN
    m = E.Model(_dims(E, d), 0, ct).init_synthetic(11)
    W = {name: m.get_tensor(name, shape) for name, shape, _, _ in O.tensor_specs(d)}
    W["encoder.embed_positions.weight"] = O.sinusoids(1500, d.n_audio_state)
    if ct == "float8":
        W = O.fp8_decoder_weights(W, d)
    heads = E.ALIGNMENT_HEADS["large-v3"]
    sp = O.special_tokens(d.n_vocab)
    ctx = E.Context(m, max_batch=2, beam_size=5, max_new_tokens=120, word_timestamps=True, alignment_heads=heads,
                    language=sp.lang0)
    audios = [synth.speech_like(821, 480000), synth.speech_like(822, 400000)]
    encs = ctx.encode(np.stack([O.logmel_segment(a, d.n_mels) for a in audios]))
    res = ctx.transcribe(audios)
    out = []
    for b, r in enumerate(res):
        text = [t for t in r.tokens if t < sp.eot]
        assert len(text) >= 100, len(text)
        dev = ctx.alignment_matrix(b)
        ti, tj = A._lib_dtw(dev)
        np.testing.assert_array_equal(r.jump_times, A._jumps(ti, tj).astype(np.float32))
        oti, otj, probs, jt, ref = O.find_alignment(W, d, encs[b], sp.lang0, "transcribe", text, r.seek_frames,
                                                     align_heads=heads, return_matrix=True)
        e = rel_l2(dev, ref)
        near = np.abs(r.jump_times - jt) <= 0.02 + 1e-6
        ex, bd, rex = A.path_check(dev, ref, ti, tj, oti, otj)
        print(f"{ct} window {b}: {len(text)} text tokens, matrix rel_l2 {e:.2e}, jump times within 1 frame "
              f"{float(np.mean(near)):.3f} ({int((~near).sum())} off), token probs max err "
              f"{float(np.max(np.abs(r.text_token_probs - probs))):.2e}; device path excess cost {ex:.4f} <= {bd:.4f}")
        np.testing.assert_allclose(r.text_token_probs, probs, atol=2e-2)
        # the relative form of path_check's bound: the summed matrix error over both paths / the oracle path's cost
        rbd = _rel_bound(ref, oti, otj, bd)
        out.append((e, float(np.mean(near)), int((~near).sum()), len(text), rex, rbd))
    return out


def _rel_bound(ref, oti, otj, bound):
    """path_check's bound relative to the oracle path's cost on the oracle's matrix (the scale rex is quoted on)."""
    cost_ref = -ref.astype(np.float64)[np.asarray(oti, np.int64), np.asarray(otj, np.int64)].sum()
    return float(bound / max(abs(cost_ref), 1e-30))


def test_fp8_decode_word_alignment_large_v3_heads():
    """The word-alignment pass of the fp8 model (the alignment forward over sot + text + eot runs its > 256-row
    projections on the dequantized row-major copies, its cross attention on the fp8 images, its logits on the 8-bit
    embedding) held to the bf16 model's numbers on the same two windows and protocol.

    * bf16 leg: tests/test_gpu_align.py's criteria -- matrix rel-L2 <= 3e-2, the device DTW path near-optimal on the
      oracle's matrix (path_check: excess cost <= the summed matrix error over both paths, exact when both DTWs are),
      and the coarse floor on jump times within one frame (test_gpu_align.WITHIN_FLOOR; the oracle's own path moves at near-ties with its BLAS
      order: this same bf16 leg gave 99.2 % on one box and 94.2 % on another with identical device matrices).
    * fp8 leg, relative to the bf16 leg window by window: matrix rel-L2 <= 1.6 x bf16's (the e4m3 K images add one
      rounding on top of bf16's: an element a 16-bit ulp from the oracle's can land on the neighbouring e4m3 code, a
      6 % step; measured 1.45-1.52 x), and the same path criterion on its OWN measured matrix error: the fp8 path's
      excess cost on the oracle's matrix <= the summed |fp8 matrix - oracle matrix| over both paths (asserted inside
      path_check, and restated here in relative form per window).
    Round 5 asserted instead `rx8 <= 2 rx16 + 1e-3`, a heuristic whose slack is a bare 1e-3 when the bf16 path is exact
    (rx16 = 0); it went red once (gpurun_out/r05p: rx8 1.61e-3, rx16 0) on a build whose GELU rounding differed by one
    ulp, while the fp8 leg's own error bound held.  The bound below is derived from the leg's measured error, so a
    1-ulp change elsewhere moves the bound with the path.
    Both legs: token probabilities within 2e-2 of the oracle's, and jump times equal to the library DTW of the device
    matrix."""
    import test_gpu_align as A
    legs = {ct: _alignment_legs(ct) for ct in ("bfloat16", "float8")}
    for b, ((e16, w16, off16, _, rx16, rb16), (e8, w8, off8, _, rx8, rb8)) in enumerate(
            zip(legs["bfloat16"], legs["float8"])):
        print(f"window {b}: fp8 / bf16 matrix rel-L2 {e8 / e16:.2f}, off by > 1 frame {off8} vs {off16}, relative "
              f"path excess {rx8:.2e} (bound {rb8:.2e}) vs bf16 {rx16:.2e} (bound {rb16:.2e})")
        assert e16 <= 3e-2, e16
        assert w16 >= A.WITHIN_FLOOR and w8 >= A.WITHIN_FLOOR, (w16, w8)
        assert e8 <= 1.6 * e16, (e8, e16)
        assert rx16 <= rb16 + 1e-4 and rx8 <= rb8 + 1e-4, (rx16, rb16, rx8, rb8)
