"""GPU parity of the decode STEP at the bench's shapes, and of the decode SEARCH over every step.

What bench.py times per decode step (wmx_runtime.hip dec_step_fast + logits + select/update, replayed from a
hipGraph) is checked here at the shapes it runs in, against the oracle, in two complementary ways:

  * Step kernels, teacher-forced (wmx_ctx_forced_decode): the rows of B windows are fed a fixed token stream
    (and, for beams, a fixed parent per row and step, i.e. the beam reorder of the ancestry rows) and the raw logits
    of every step are compared with oracle.forced_rows (openai BeamSearchDecoder semantics: a new row continues its
    parent's KV cache).  Shapes: large-v3 width (d = 1280, 20 heads, 128 mels, vocab 51866) with 20 rows -- the
    per-group rows of the bench (4 windows x beam 5 and 20 windows greedy): packed split-K GEMMs with two 16-row
    fragments (MT = 2), fc2 over K = 5120, the 16-wave fc1 -- and a micro model over 224 steps, so the
    ancestry-gathered self attention runs past slot 200 with beams reordered every step.
    Tolerances: relative L2 of each row's logits, bf16 <= 3e-2, f16 <= 5e-3 (tests/test_gpu_parity.py); and the
    argmax must equal the oracle's wherever the oracle's top-2 margin exceeds twice the row's measured max abs
    error (then no error of that size can flip it).  The number of steps compared this way is printed, and
    f16 requires >= 16 per row.
  * Search, token-exact (wmx_ctx_record + oracle.search_replay): a free-running transcribe records every step's
    raw logits and the device's selection; the oracle replays the rules, top-k, beam bookkeeping and finished
    handling on those same logits and must choose exactly the device's (parent, token) at every step (a step whose
    deciding score gap is below 1e-3 is a legitimate f32-vs-f64 tie and ends that window's comparison), and the
    final ranked sequence must equal the device's result.  This is what makes beam-5 parity testable at all with
    random weights: free-running beams on random weights sit on near-ties (tools/ notes in DESIGN.md §4).
"""
import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

pytestmark = pytest.mark.gpu

WIDE2 = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 2)  # large-v3 width, 1 encoder layer, 2 decoder layers
REL = {"bf16": 3e-2, "f16": 5e-3}
DT = {"bf16": "bfloat16", "f16": "float16"}
EPS_TIE = 1e-3


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _edims(d):
    from wmx import engine as E
    return E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                       d.n_text_head, d.n_text_layer)


def _forced_stream(rng, n, R, K, V=50000):
    tok = rng.integers(0, V, size=(n, R)).astype(np.int32)
    par = np.tile(np.arange(R, dtype=np.int32), (n, 1))
    if K > 1:
        for i in range(n):
            for b in range(R // K):
                par[i, b * K:(b + 1) * K] = b * K + rng.integers(0, K, size=K)
    return tok, par


def _check_forced(tag, dt, top1, lg, every, ref_top1, ref_margin, ref_lg, min_cmp):
    """rel-L2 at every snapshot step and argmax equality wherever the oracle margin > 2 x the row's max error."""
    n1, R = top1.shape
    err_row = np.zeros(R)
    worst = 0.0
    for si, step in enumerate(range(0, n1, every)):
        for r in range(R):
            e = rel_l2(lg[si, r], ref_lg[step][r])
            worst = max(worst, e)
            assert e <= REL[dt], (tag, step, r, e)
            err_row[r] = max(err_row[r], float(np.max(np.abs(lg[si, r] - ref_lg[step][r]))))
    cmp = np.zeros(R, int)
    for r in range(R):
        # steps without a logits snapshot use the row's worst snapshot error, x1.5
        tau = 2 * err_row[r] * (1.0 if every == 1 else 1.5)
        sel = ref_margin[:, r] > tau
        np.testing.assert_array_equal(top1[sel, r], ref_top1[sel, r], err_msg=f"{tag} row {r}")
        cmp[r] = int(sel.sum())
    print(f"{tag} {dt}: {n1} steps x {R} rows, worst rel_l2 {worst:.2e}, argmax compared per row "
          f"min {cmp.min()} mean {cmp.mean():.1f} of {n1}")
    if dt == "f16":
        assert cmp.min() >= min_cmp, cmp


# ---------------------------------------------------------------------------------------------------------------
# large-v3 width fixture: 20 windows encoded once per dtype
# ---------------------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module", params=["bf16", "f16"])
def wide20(request):
    from wmx import engine as E
    dt = request.param
    m = E.Model(_edims(WIDE2), 0, DT[dt]).init_synthetic(5)
    W = O.make_weights(WIDE2, 5, dt)
    lens = [480000, 150000, 320000, 16000, 240000] * 4
    mels = np.stack([O.logmel_segment(synth.speech_like(100 + i, n), 128) for i, n in enumerate(lens)])
    encs = [O.encoder(W, WIDE2, mel) for mel in mels]
    return dt, m, W, mels, encs


def test_forced_steps_wide_20rows_greedy(wide20):
    """20 windows x greedy = 20 decode rows at d = 1280 (the bench's per-group row count), 32 forced steps."""
    from wmx import engine as E
    dt, m, W, mels, encs = wide20
    sp = O.special_tokens(WIDE2.n_vocab)
    ctx = E.Context(m, max_batch=20, beam_size=1, max_new_tokens=64, word_timestamps=False)
    ctx.encode(mels, want_output=False)
    n = 32
    tok, par = _forced_stream(np.random.default_rng(1), n, 20, 1)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]] * 20
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, WIDE2, encs, prefix, tok, par, 1)
    _check_forced("wide greedy R=20", dt, top1, lg, 1, ref_top1, ref_margin, ref_lg, 16)


def test_forced_steps_wide_beam5_4windows(wide20):
    """4 windows x beam 5 = 20 rows, parents re-drawn every step (ancestry-gathered self attention at width)."""
    from wmx import engine as E
    dt, m, W, mels, encs = wide20
    sp = O.special_tokens(WIDE2.n_vocab)
    ctx = E.Context(m, max_batch=4, beam_size=5, max_new_tokens=64, word_timestamps=False)
    ctx.encode(mels[:4], want_output=False)
    n = 32
    tok, par = _forced_stream(np.random.default_rng(2), n, 20, 5)
    # a prompted batch: previous-text prompts of different lengths, left-padded together (transcribe's layout)
    prefix = [[sp.sot_prev] + list(range(1000, 1000 + L)) + [sp.sot, sp.lang0, sp.transcribe] for L in (0, 5, 11, 2)]
    prefix[0] = [sp.sot, sp.lang0, sp.transcribe]
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, WIDE2, encs[:4], prefix, tok, par, 5)
    _check_forced("wide beam5 B=4", dt, top1, lg, 1, ref_top1, ref_margin, ref_lg, 16)


def test_forced_steps_micro_beam5_224():
    """224 steps with beams reordered every step: self attention over up to 227 ancestry-gathered slots."""
    from wmx import engine as E
    d = O.DIMS["micro"]
    sp = O.special_tokens(d.n_vocab)
    dt = "f16"
    m = E.Model("micro", 0, DT[dt]).init_synthetic(1)
    W = O.make_weights(d, 1, dt)
    mels = np.stack([O.logmel_segment(synth.speech_like(200 + i, n), 80)
                     for i, n in enumerate((480000, 200000, 96000, 330000))])
    encs = [O.encoder(W, d, mel) for mel in mels]
    ctx = E.Context(m, max_batch=4, beam_size=5, max_new_tokens=224, word_timestamps=False)
    ctx.encode(mels, want_output=False)
    n, every = 224, 8
    tok, par = _forced_stream(np.random.default_rng(3), n, 20, 5)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]] * 4
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=every)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, d, encs, prefix, tok, par, 5, keep=range(0, n + 1, every))
    _check_forced("micro beam5 224 steps", dt, top1, lg, every, ref_top1, ref_margin, ref_lg, 150)


# ---------------------------------------------------------------------------------------------------------------
# search parity: free-running transcribe, recorded, replayed by the oracle
# ---------------------------------------------------------------------------------------------------------------
def _replay_and_compare(tag, ctx, res, K, opt, sp, min_steps):
    lg, sel = ctx.recorded()
    info = O.search_replay(lg, sel, K, sp, opt, eps=EPS_TIE)
    steps = []
    for b, (r, inf) in enumerate(zip(res, info)):
        assert inf["mismatch"] is None, (tag, b, inf["mismatch"])
        steps.append(inf["steps"])
        if inf["ties"]:
            continue
        if K == 1:
            ref = inf["finished"][0][0] if inf["finished"] else inf["alive"][0][0]
            assert r.tokens == ref, (tag, b, r.tokens, ref)
        else:
            toks, sc, margin = O.rank_final(inf["finished"], inf["alive"], K)
            if margin > EPS_TIE:
                assert r.tokens == toks, (tag, b, r.tokens, toks)
                assert abs(r.sum_logprob - sc) <= 1e-3 * max(1.0, abs(sc)), (tag, b, r.sum_logprob, sc)
    ties = sum(i["ties"] for i in info)
    ran = [int((sel[:, b * K, 0] >= 0).sum()) for b in range(len(res))]  # steps the device searched per window
    print(f"{tag}: recorded {lg.shape[0]} steps x {lg.shape[1]} rows; replayed steps per window {steps} "
          f"(device ran {ran}); windows ended by a float tie {ties}")
    short = [b for b in range(len(res)) if not info[b]["ties"] and steps[b] < min(min_steps, ran[b])]
    assert not short, (short, steps, ran)
    return info


def test_search_replay_wide_greedy_20windows(wide20):
    from wmx import engine as E
    dt, m, W, mels, encs = wide20
    sp = O.special_tokens(WIDE2.n_vocab)
    audios = [synth.speech_like(100 + i, n) for i, n in enumerate([480000, 150000, 320000, 16000, 240000] * 4)]
    ctx = E.Context(m, max_batch=20, beam_size=1, max_new_tokens=32, word_timestamps=False)
    ctx.record(33)
    res = ctx.transcribe(audios)
    langs = {r.language for r in res}
    for b in (0, 3):  # language detection vs the oracle (the replay starts after it)
        assert res[b].language == O.detect_language(W, WIDE2, encs[b])[0]
    opt = O.DecodeOptions(beam_size=1, max_new_tokens=32)
    _replay_and_compare(f"wide greedy B=20 {dt} (langs {sorted(langs)})", ctx, res, 1, opt, sp, 16)


def test_search_replay_wide_beam5_4windows(wide20):
    from wmx import engine as E
    dt, m, W, mels, encs = wide20
    sp = O.special_tokens(WIDE2.n_vocab)
    audios = [synth.speech_like(100 + i, n) for i, n in enumerate([480000, 150000, 320000, 16000])]
    ctx = E.Context(m, max_batch=4, beam_size=5, max_new_tokens=32, word_timestamps=False, language=sp.lang0)
    ctx.record(33)
    res = ctx.transcribe(audios, prompts=[[], [1000, 1001, 1002], [2000 + i for i in range(9)], [5]])
    opt = O.DecodeOptions(language=sp.lang0, beam_size=5, max_new_tokens=32)
    _replay_and_compare(f"wide beam5 B=4 prompted {dt}", ctx, res, 5, opt, sp, 16)


@pytest.mark.parametrize("K", [1, 5])
def test_search_replay_micro_224_steps(K):
    """The whole 224-step decode of the bench's max_new_tokens, greedy and beam 5, replayed exactly."""
    from wmx import engine as E
    d = O.DIMS["micro"]
    sp = O.special_tokens(d.n_vocab)
    m = E.Model("micro", 0, "bfloat16").init_synthetic(1)
    ctx = E.Context(m, max_batch=2, beam_size=K, max_new_tokens=224, word_timestamps=False, language=sp.lang0)
    ctx.record(224)
    res = ctx.transcribe([synth.speech_like(301, 480000), synth.speech_like(302, 200000)])
    opt = O.DecodeOptions(language=sp.lang0, beam_size=K, max_new_tokens=224)
    _replay_and_compare(f"micro K={K} 224 steps", ctx, res, K, opt, sp, 100)
    ctx.record(0)


def test_recorder_off_keeps_results():
    """The recorder's launches change nothing: same tokens with it on and off (graph re-captured each way)."""
    from wmx import engine as E
    m = E.Model("micro", 0, "bfloat16").init_synthetic(1)
    ctx = E.Context(m, max_batch=2, beam_size=5, max_new_tokens=40, word_timestamps=True)
    audios = [synth.speech_like(401, 300000), synth.speech_like(402, 100000)]
    a = ctx.transcribe(audios)
    ctx.record(40)
    b = ctx.transcribe(audios)
    ctx.record(0)
    c = ctx.transcribe(audios)
    for x, y, z in zip(a, b, c):
        assert x.tokens == y.tokens == z.tokens


# ---------------------------------------------------------------------------------------------------------------
# full depth: the real large-v3 (32 + 32 layers), one window
# ---------------------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def large_v3():
    """The real large-v3 (32 + 32 layers, bf16, PRNG weights) and the oracle's copy of its weights: read back from the
    device (bit-exact with O.make_weights: test_weights_bit_exact; the numpy PRNG over 1.55 B parameters would take a
    minute), as bench.py's cpu_baseline does."""
    from wmx import engine as E
    d = O.DIMS["large-v3"]
    m = E.Model("large-v3", 0, "bfloat16").init_synthetic(1)
    W = {name: m.get_tensor(name, shape) for name, shape, _, _ in O.tensor_specs(d)}
    W["encoder.embed_positions.weight"] = O.sinusoids(1500, d.n_audio_state)
    ref_small = O.make_weights(O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 1), 1, "bf16")
    np.testing.assert_array_equal(W["encoder.layers.0.fc1.weight"], ref_small["encoder.layers.0.fc1.weight"])
    return m, W


def test_full_depth_large_v3_one_window(large_v3):
    """Encoder rel-L2 over all 32 layers and 8 forced decode steps through all 32 decoder layers (bf16), plus the
    first free-running greedy steps replayed exactly."""
    from wmx import engine as E
    d = O.DIMS["large-v3"]
    sp = O.special_tokens(d.n_vocab)
    dt = "bf16"
    m, W = large_v3
    audio = synth.speech_like(501, 480000)
    mel = O.logmel_segment(audio, d.n_mels)
    enc = O.encoder(W, d, mel)
    ctx = E.Context(m, max_batch=1, beam_size=1, max_new_tokens=8, word_timestamps=False, language=sp.lang0)
    got = ctx.encode(mel[None])[0]
    e = rel_l2(got, enc)
    print("large-v3 full-depth encoder rel_l2", e)
    assert e <= REL[dt], e
    n = 8
    tok, par = _forced_stream(np.random.default_rng(4), n, 1, 1)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]]
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, d, [enc], prefix, tok, par, 1)
    _check_forced("large-v3 full depth", dt, top1, lg, 1, ref_top1, ref_margin, ref_lg, 0)
    ctx.record(8)
    res = ctx.transcribe([audio])
    opt = O.DecodeOptions(language=sp.lang0, beam_size=1, max_new_tokens=8)
    _replay_and_compare("large-v3 full depth greedy", ctx, res, 1, opt, sp, 1)


def test_full_depth_large_v3_encoder_layernorm_fold(large_v3):
    """The encoder with its LayerNorms folded into qkv / fc1 (Model::enc_fold, on from 4096 rows: 3 windows here), all
    32 layers, against the oracle's unfolded fp32 LayerNorms; and against the same device model with the fold off
    (WMX_ENC_FOLD=0, read at model creation) -- the fold's own numerical cost, bf16."""
    import os
    from wmx import engine as E
    d = O.DIMS["large-v3"]
    m, W = large_v3
    audios = [synth.speech_like(521, 480000), synth.speech_like(522, 300000), synth.speech_like(523, 480000)]
    mels = np.stack([O.logmel_segment(a, d.n_mels) for a in audios])
    ctx = E.Context(m, max_batch=3, beam_size=1, max_new_tokens=8, word_timestamps=False)
    got = ctx.encode(mels)
    os.environ["WMX_ENC_FOLD"] = "0"
    try:
        m0 = E.Model("large-v3", 0, "bfloat16").init_synthetic(1)
    finally:
        del os.environ["WMX_ENC_FOLD"]
    ctx0 = E.Context(m0, max_batch=3, beam_size=1, max_new_tokens=8, word_timestamps=False)
    got0 = ctx0.encode(mels)
    for b in (0, 1):
        ref = O.encoder(W, d, mels[b])
        e, e0, ef = rel_l2(got[b], ref), rel_l2(got0[b], ref), rel_l2(got[b], got0[b])
        print(f"large-v3 encoder window {b}: folded rel_l2 {e:.3e}, unfolded {e0:.3e}, folded vs unfolded {ef:.3e}")
        assert e <= REL["bf16"], e
        assert e <= 3 * e0 + 2e-3, (e, e0)  # the fold may not dominate the error budget
    del ctx0
    m0.close()


def test_full_depth_large_v3_beam5_two_windows(large_v3):
    """Beam 5 (the reference default, asr_components.py:282; BASELINE config 3) through all 32 + 32 layers: 2 windows x
    5 rows, 16 teacher-forced steps with the beams re-parented every step (every row's logits vs the oracle), then a
    free-running 16-step beam-5 transcribe replayed token-exact by oracle.search_replay / rank_final."""
    from wmx import engine as E
    d = O.DIMS["large-v3"]
    sp = O.special_tokens(d.n_vocab)
    m, W = large_v3
    audios = [synth.speech_like(511, 480000), synth.speech_like(512, 260000)]
    mels = np.stack([O.logmel_segment(a, d.n_mels) for a in audios])
    encs = [O.encoder(W, d, mel) for mel in mels]
    ctx = E.Context(m, max_batch=2, beam_size=5, max_new_tokens=16, word_timestamps=False, language=sp.lang0)
    ctx.encode(mels, want_output=False)
    n = 16
    tok, par = _forced_stream(np.random.default_rng(14), n, 10, 5)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]] * 2
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, d, encs, prefix, tok, par, 5)
    _check_forced("large-v3 full depth beam5", "bf16", top1, lg, 1, ref_top1, ref_margin, ref_lg, 0)
    ctx.record(16)
    res = ctx.transcribe(audios)
    opt = O.DecodeOptions(language=sp.lang0, beam_size=5, max_new_tokens=16)
    _replay_and_compare("large-v3 full depth beam5", ctx, res, 5, opt, sp, 8)


def _boost_eot(m, d, factor):
    """Scale the EOT embedding row (tied to the output projection) so that EOT competes in the top-k and beams finish:
    finished-hypothesis handling, patience and the length-penalised ranking only act once hypotheses end."""
    sp = O.special_tokens(d.n_vocab)
    emb = m.get_tensor("decoder.embed_tokens.weight", (d.n_vocab, d.n_text_state))
    emb[sp.eot] *= factor
    m.set_tensor("decoder.embed_tokens.weight", emb)
    m.mark_loaded()


@pytest.mark.parametrize("patience,length_penalty", [(2.0, 0.5), (1.5, None), (1.0, 1.2)])
def test_beam_options_replay_micro(patience, length_penalty):
    """Non-default faster-whisper beam options (TranscriptionOptions.patience / length_penalty, carried in wmx_opts)
    on the device, with EOT made likely so that hypotheses finish: every step's selection and the final ranking
    replayed by oracle.search_replay / rank_final with the same options."""
    from wmx import engine as E
    d = O.DIMS["micro"]
    sp = O.special_tokens(d.n_vocab)
    K = 5
    audios = [synth.speech_like(1201 + i, n) for i, n in enumerate((480000, 200000, 90000))]
    opt = O.DecodeOptions(language=sp.lang0, beam_size=K, patience=patience, length_penalty=length_penalty,
                          max_new_tokens=64)
    # EOT made competitive: its embedding row (tied to the output projection) becomes a scaled copy of the row of the
    # token the un-modified beams repeat (random weights lock onto one token), so EOT enters the top K + 1 candidates
    # and hypotheses finish; the first scale of a fixed ladder at which some hypothesis finishes is used
    m = E.Model("micro", 0, "bfloat16").init_synthetic(1)
    ctx = E.Context(m, max_batch=3, beam_size=K, max_new_tokens=16, word_timestamps=False, language=sp.lang0)
    toks0 = [t for r in ctx.transcribe(audios) for t in r.tokens if t < sp.eot]
    top = int(np.bincount(toks0).argmax())
    emb0 = m.get_tensor("decoder.embed_tokens.weight", (d.n_vocab, d.n_text_state))
    for factor in (0.9, 0.97, 1.02):
        emb = emb0.copy()
        emb[sp.eot] = factor * emb0[top]
        m.set_tensor("decoder.embed_tokens.weight", emb)
        m.mark_loaded()
        ctx = E.Context(m, max_batch=3, beam_size=K, patience=patience,
                        length_penalty=1.0 if length_penalty is None else length_penalty, max_new_tokens=64,
                        word_timestamps=False, language=sp.lang0)
        ctx.record(64)
        res = ctx.transcribe(audios)
        lg, sel = ctx.recorded()
        info = O.search_replay(lg, sel, K, sp, opt, eps=EPS_TIE)
        fin = [len(i["finished"]) for i in info]
        if sum(fin) > 0:
            break
    for b, (r, inf) in enumerate(zip(res, info)):
        assert inf["mismatch"] is None, (b, inf["mismatch"])
        if inf["ties"]:
            continue
        toks, sc, margin = O.rank_final(inf["finished"], inf["alive"], K, length_penalty)
        if margin > EPS_TIE:
            assert r.tokens == toks, (b, r.tokens, toks)
            assert abs(r.sum_logprob - sc) <= 1e-3 * max(1.0, abs(sc)), (b, r.sum_logprob, sc)
    print(f"patience {patience} length_penalty {length_penalty} (EOT = {factor} x row {top}): replayed "
          f"{[i['steps'] for i in info]} steps, finished hypotheses per window {fin}, token counts "
          f"{[len(r.tokens) for r in res]}")
    assert sum(fin) > 0  # the options were exercised: hypotheses did finish
    assert max(fin) <= int(round(K * patience))


def test_beam_options_replay_wide():
    """The same at large-v3 width (d 1280, vocab 51866, 4 windows x beam 5 = the bench group's 20 rows), patience 2,
    length penalty 0.5."""
    from wmx import engine as E
    sp = O.special_tokens(WIDE2.n_vocab)
    m = E.Model(_edims(WIDE2), 0, "bfloat16").init_synthetic(5)
    _boost_eot(m, WIDE2, 4.0)
    K, n_new = 5, 48
    ctx = E.Context(m, max_batch=4, beam_size=K, patience=2.0, length_penalty=0.5, max_new_tokens=n_new,
                    word_timestamps=False, language=sp.lang0)
    ctx.record(n_new)
    audios = [synth.speech_like(100 + i, n) for i, n in enumerate([480000, 150000, 320000, 16000])]
    res = ctx.transcribe(audios)
    opt = O.DecodeOptions(language=sp.lang0, beam_size=K, patience=2.0, length_penalty=0.5, max_new_tokens=n_new)
    lg, sel = ctx.recorded()
    info = O.search_replay(lg, sel, K, sp, opt, eps=EPS_TIE)
    fin = [len(i["finished"]) for i in info]
    for b, (r, inf) in enumerate(zip(res, info)):
        assert inf["mismatch"] is None, (b, inf["mismatch"])
        if inf["ties"]:
            continue
        toks, sc, margin = O.rank_final(inf["finished"], inf["alive"], K, 0.5)
        if margin > EPS_TIE:
            assert r.tokens == toks, (b, r.tokens, toks)
    print(f"wide patience 2 lp 0.5: replayed {[i['steps'] for i in info]}, finished per window {fin}")
    assert sum(fin) > 0


def test_control_tokens_suppressed_with_boosted_logits():
    """faster-whisper / openai always suppress the task / sot / prev / lm / no_speech ids (tokenizer.suppressed_tokens).
    Their embedding rows are boosted so they would win every step; with the adapter's suppress list they are never
    chosen (and the replay checks the device's mask step by step); without it they are (so the test has teeth)."""
    from wmx import engine as E
    from wmx.tokenizer import SpecialTokens, suppressed_tokens
    d = O.DIMS["micro"]
    sp = O.special_tokens(d.n_vocab)
    ctrl = [sp.transcribe, sp.translate, sp.sot, sp.sot_prev, sp.sot_lm, sp.no_speech]
    m = E.Model("micro", 0, "bfloat16").init_synthetic(1)
    emb = m.get_tensor("decoder.embed_tokens.weight", (d.n_vocab, d.n_text_state))
    emb[ctrl] *= 40.0
    m.set_tensor("decoder.embed_tokens.weight", emb)
    sup = suppressed_tokens(SpecialTokens(d.n_vocab))
    assert set(ctrl) <= set(sup)
    audios = [synth.speech_like(601, 240000), synth.speech_like(602, 90000)]
    for K in (1, 5):
        ctx = E.Context(m, max_batch=2, beam_size=K, max_new_tokens=24, word_timestamps=False, language=sp.lang0,
                        suppress_tokens=sup)
        ctx.record(24)
        res = ctx.transcribe(audios)
        for r in res:
            assert not set(r.tokens) & set(ctrl), r.tokens
        opt = O.DecodeOptions(language=sp.lang0, beam_size=K, max_new_tokens=24, suppress_tokens=tuple(sup))
        _replay_and_compare(f"suppressed control tokens K={K}", ctx, res, K, opt, sp, 16)
        bare = E.Context(m, max_batch=2, beam_size=K, max_new_tokens=24, word_timestamps=False, language=sp.lang0)
        assert any(set(r.tokens) & set(ctrl) for r in bare.transcribe(audios))


def test_separate_cross_q_step_parity():
    """The decode step with the cross-q projection as its own split-K launch (WMX_XQ_FUSED=0) instead of inside the
    cross attention (the default, wmx_attn.hip dec_cross_attn_kernel<..., XQ = true>): the teacher-forced step tests
    of this file in a child process with the switch set (read at context creation)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WMX_XQ_FUSED="0")
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
           "-k", "forced_steps", "tests/test_gpu_step.py"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.timeout(900)
def test_fast_step_parity():
    """The fast decode step (WMX_DEC_MIXED=0, wmx_runtime.hip dec_step_fast: every d x d projection split-K with a
    reduce_ln launch after the out-projection, the cross out-projection and fc2).  The mixed step (dec_step_mixed: the
    out-projection and the cross out-projection unsplit with row statistics, LN2 folded into the fused cross-q
    projection of the cross attention, LN3 into fc1's GELU epilogue) is the default for 16-bit models since round 6,
    so the rest of this file runs on it; here its step, search and full-depth tests rerun in a child process on the
    fast step (the switch is read at model creation)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WMX_DEC_MIXED="0")
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
           "-k", "not fast_step and not separate_cross_q",
           "tests/test_gpu_step.py"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=880)
    print(r.stdout[-1500:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


# ---------------------------------------------------------------------------------------------------------------
# BASELINE config 1 on the HIP path: Whisper tiny at full depth (4 + 4 layers, d 384, 80 mels), greedy
# ---------------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name,dt", [("tiny", "f16"), ("tiny", "bf16"), ("base", "f16")])
def test_full_depth_small_models_greedy(name, dt):
    """Config 1's model (tiny) and config 2's (base, fp16) through the whole HIP path at full depth: encoder rel-L2,
    language detection, 24 forced decode steps over 3 windows (every row's logits every step) and the free-running
    greedy search replayed token-exact."""
    from wmx import engine as E
    d = O.DIMS[name]
    sp = O.special_tokens(d.n_vocab)
    m = E.Model(name, 0, DT[dt]).init_synthetic(3)
    W = O.make_weights(d, 3, dt)
    lens = [480000, 200000, 64000]
    audios = [synth.speech_like(700 + i, n) for i, n in enumerate(lens)]
    mels = np.stack([O.logmel_segment(a, d.n_mels) for a in audios])
    encs = [O.encoder(W, d, mel) for mel in mels]
    ctx = E.Context(m, max_batch=3, beam_size=1, max_new_tokens=48, word_timestamps=False)
    got = ctx.encode(mels)
    for b in range(3):
        e = rel_l2(got[b], encs[b])
        assert e <= REL[dt], (b, e)
    n = 24
    tok, par = _forced_stream(np.random.default_rng(9), n, 3, 1)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]] * 3
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(W, d, encs, prefix, tok, par, 1)
    _check_forced(f"{name} full depth", dt, top1, lg, 1, ref_top1, ref_margin, ref_lg, 16)
    ctx.record(49)
    res = ctx.transcribe(audios)
    for b in range(3):
        assert res[b].language == O.detect_language(W, d, encs[b])[0]
    opt = O.DecodeOptions(beam_size=1, max_new_tokens=48)
    _replay_and_compare(f"{name} full depth greedy {dt}", ctx, res, 1, opt, sp, 24)


# ---------------------------------------------------------------------------------------------------------------
# temperature > 0 (faster-whisper's sampling branch; the reference's speech-rate adaptation sets T = 0.1,
# speech_rate_audio_processor.py:217-218): best_of rows per window drawn by Gumbel-max, replayed by the oracle with
# the same counter-based noise (oracle.sample_gumbel); parity with CT2's own random draws is unpinned by nature
# ---------------------------------------------------------------------------------------------------------------
def _sampling_replay_and_compare(tag, ctx, res, K, opt, sp, T, seed, min_steps):
    lg, sel = ctx.recorded()
    info = O.sampling_replay(lg, sel, K, sp, opt, T, seed, slot0=2, eps=EPS_TIE)
    steps, ties, distinct = [], 0, []
    for b, (r, inf) in enumerate(zip(res, info)):
        for j, rw in enumerate(inf["rows"]):
            assert rw["mismatch"] is None, (tag, b, j, rw["mismatch"])
            steps.append(rw["steps"])
            ties += rw["ties"]
        distinct.append(len({tuple(rw["tokens"]) for rw in inf["rows"]}))
        if inf["best"] is not None:
            _, toks, total = inf["best"]
            assert r.tokens == toks, (tag, b, r.tokens, toks)
            assert abs(r.sum_logprob - total) <= 1e-3 * max(1.0, abs(total)), (tag, b, r.sum_logprob, total)
    print(f"{tag}: replayed steps per row {steps}; rows ended by a float tie {ties}; distinct samples per window "
          f"{distinct}")
    assert min(s for s in steps) >= min(min_steps, 1) and sum(steps) >= min_steps * len(steps) // 2
    return info, distinct


def test_sampling_replay_micro():
    from wmx import engine as E
    d = O.DIMS["micro"]
    sp = O.special_tokens(d.n_vocab)
    m = E.Model("micro", 0, "bfloat16").init_synthetic(1)
    T, seed = 1.0, 1234
    ctx = E.Context(m, max_batch=3, beam_size=7, max_new_tokens=64, word_timestamps=True, language=sp.lang0,
                    temperature=T, best_of=4, sample_seed=seed)
    ctx.record(64)
    res = ctx.transcribe([synth.speech_like(501, 480000), synth.speech_like(502, 160000), synth.speech_like(503, 32000)])
    opt = O.DecodeOptions(language=sp.lang0, beam_size=1, max_new_tokens=64)
    _, distinct = _sampling_replay_and_compare("micro T=1.0 best_of 4", ctx, res, 4, opt, sp, T, seed, 16)
    assert max(distinct) > 1  # the rows of a window are independent draws
    assert all(r.jump_times is not None for r in res)  # word alignment runs on the chosen row


def test_sampling_replay_wide_adaptive_shape(wide20):
    """The reference's fast-speech setting (beam 7, T 0.1 -> faster-whisper samples best_of = 5) at large-v3 width:
    4 windows x 5 rows, prompted."""
    from wmx import engine as E
    dt, m, W, mels, encs = wide20
    sp = O.special_tokens(WIDE2.n_vocab)
    T, seed = 0.1, 99
    ctx = E.Context(m, max_batch=4, beam_size=7, max_new_tokens=32, word_timestamps=False, language=sp.lang0,
                    temperature=T, best_of=5, sample_seed=seed)
    ctx.record(33)
    audios = [synth.speech_like(100 + i, n) for i, n in enumerate([480000, 150000, 320000, 16000])]
    res = ctx.transcribe(audios)
    opt = O.DecodeOptions(language=sp.lang0, beam_size=1, max_new_tokens=32)
    _sampling_replay_and_compare(f"wide T=0.1 best_of 5 {dt}", ctx, res, 5, opt, sp, T, seed, 16)
