"""Pin the CPU oracle against the committed golden fixtures (transformers 5.15.0, see tests/golden/make_golden.py)."""
import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

AUDIO = {
    "sp_0p5": ("speech", 11, 0.5), "sp_1": ("speech", 12, 1.0), "sp_7p3": ("speech", 13, 7.3),
    "noise_4": ("noise", 14, 4.0), "zeros_2": ("zeros", 0, 2.0), "sp_30": ("speech", 15, 30.0),
    "sp_31": ("speech", 16, 31.0),
}


def make_audio(kind, seed, sec):
    n = int(round(sec * 16000))
    if kind == "speech":
        return synth.speech_like(seed, n)
    if kind == "noise":
        return synth.white_noise(seed, n)
    return np.zeros(n, np.float32)


@pytest.mark.parametrize("name", list(AUDIO))
@pytest.mark.parametrize("n_mels", [80, 128])
def test_logmel_matches_golden(golden, name, n_mels):
    a = make_audio(*AUDIO[name])
    assert synth.digest(a) == bytes(golden[f"logmel/{name}/sha"]).decode(), "synthetic audio generator drifted"
    ref = golden[f"logmel/{name}/{n_mels}/value"]
    idx = golden[f"logmel/{name}/{n_mels}/frames"]
    got = O.logmel(a, n_mels)
    assert got.shape[1] == int(golden[f"logmel/{name}/{n_mels}/nframes"]) == len(a) // 160 + 1
    np.testing.assert_allclose(got[:, idx], ref, atol=1e-4, rtol=0)


def test_logmel_segment_padding():
    a = synth.speech_like(3, 16000 * 5)
    seg = O.logmel_segment(a, 80)
    feats = O.logmel(a, 80)
    assert seg.shape == (80, 3000)
    np.testing.assert_array_equal(seg[:, :500], feats[:, :500])  # content_frames = F - 1 = 500
    assert np.all(seg[:, 500:] == 0.0)
    a30 = synth.speech_like(4, 480000)
    np.testing.assert_array_equal(O.logmel_segment(a30, 80), O.logmel(a30, 80)[:, :3000])


def test_reflect_index_matches_numpy_pad():
    for n in (1, 2, 3, 7, 50):
        x = np.arange(n, dtype=np.float64)
        pad = 130
        ref = np.pad(x, (pad, pad), mode="reflect") if n > 1 else np.full(n + 2 * pad, x[0])
        got = x[O.reflect_index(np.arange(-pad, n + pad), n)]
        np.testing.assert_array_equal(got, ref)


MODELS = [("micro", 1, "bf16"), ("tiny", 2, "bf16"), ("tiny", 3, "f16")]


@pytest.fixture(scope="module")
def models():
    cache = {}

    def get(name, seed, dtype):
        k = (name, seed, dtype)
        if k not in cache:
            d = O.DIMS[name]
            W = O.make_weights(d, seed, dtype)
            mel = O.logmel_segment(synth.speech_like(21, int(round(7.3 * 16000))), d.n_mels)
            cache[k] = (d, W, O.encoder(W, d, mel))
        return cache[k]
    return get


@pytest.mark.parametrize("name,seed,dtype", MODELS)
def test_encoder_matches_golden(golden, models, name, seed, dtype):
    d, W, enc = models(name, seed, dtype)
    key = f"model/{name}/{dtype}/{seed}"
    np.testing.assert_allclose(enc[golden[key + "/enc_rows"]], golden[key + "/enc"], atol=2e-3, rtol=1e-3)


@pytest.mark.parametrize("name,seed,dtype", MODELS)
def test_decoder_logits_match_golden(golden, models, name, seed, dtype):
    d, W, _ = models(name, seed, dtype)
    key = f"model/{name}/{dtype}/{seed}"
    # feed the golden encoder rows? No: use the oracle encoder (pinned above) for the full 1500 rows.
    enc = models(name, seed, dtype)[2]
    toks = list(golden[key + "/dec_tokens"])
    cache = O.DecoderCache(W, d, enc)
    logits = O.decoder_forward(W, d, toks, cache)
    np.testing.assert_allclose(logits[:, golden[key + "/dec_probe"]], golden[key + "/dec_logits_probe"], atol=5e-3, rtol=1e-3)
    np.testing.assert_array_equal(logits.argmax(-1), golden[key + "/dec_argmax"])


@pytest.mark.parametrize("name,seed,dtype", MODELS[:1])
def test_decoder_incremental_equals_prefill(models, name, seed, dtype):
    d, W, enc = models(name, seed, dtype)
    sp = O.special_tokens(d.n_vocab)
    toks = [sp.sot, sp.lang0, sp.transcribe, sp.timestamp_begin, 400, 500]
    full = O.decoder_forward(W, d, toks, O.DecoderCache(W, d, enc))
    c = O.DecoderCache(W, d, enc)
    inc = np.concatenate([O.decoder_forward(W, d, [t], c) for t in toks])
    np.testing.assert_allclose(inc, full, atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("V", [51865, 51866])
def test_rules_match_golden(golden, V):
    sp = O.special_tokens(V)
    suppress = tuple(int(t) for t in golden[f"rules/{V}/suppress"])
    opt = O.DecodeOptions(suppress_tokens=suppress)
    n = 0
    for i in range(8):
        for variant in range(2):
            k = f"rules/{V}/{i}/{variant}"
            hist = [int(t) for t in golden[k + "/hist"] if t >= 0]
            logits = golden[k + "/logits"].astype(np.float32)
            ref = np.unpackbits(golden[k + "/masked"])[:V].astype(bool)
            got = np.isneginf(O.apply_rules(logits, hist, sp, opt))
            np.testing.assert_array_equal(got, ref, err_msg=f"{k} hist={hist}")
            n += 1
    assert n == 16


def test_dtw_matches_golden(golden):
    for i in range(4):
        ti, tj = O.dtw(golden[f"dtw/{i}/x"])
        np.testing.assert_array_equal(ti, golden[f"dtw/{i}/ti"])
        np.testing.assert_array_equal(tj, golden[f"dtw/{i}/tj"])


def test_median_filter_matches_golden(golden):
    for i in range(2):
        np.testing.assert_allclose(O.median_filter(golden[f"medfilt/{i}/x"], 7), golden[f"medfilt/{i}/y"], atol=0)


def test_special_tokens():
    s3 = O.special_tokens(51866)
    assert (s3.transcribe, s3.no_timestamps, s3.timestamp_begin) == (50360, 50364, 50365)
    s2 = O.special_tokens(51865)
    assert (s2.translate, s2.sot_prev, s2.timestamp_begin) == (50358, 50361, 50364)
    assert s2.timestamp_begin + 1500 == 51864 and s3.timestamp_begin + 1500 == 51865


def test_prng_is_exact_and_deterministic():
    u = O.prng_uniform(7, 3, 1000)
    assert u.dtype == np.float32 and u.min() >= -1.0 and u.max() < 1.0
    np.testing.assert_array_equal(u, O.prng_uniform(7, 3, 1000))
    assert not np.array_equal(u, O.prng_uniform(7, 4, 1000))
    # known-answer vector: locks the generator so the HIP init kernel and the oracle cannot drift together
    assert O.prng_uniform(1, 0, 4).tolist() == [0.7666215896606445, 0.13312304019927979, 0.1823793649673462,
                                                -0.773099422454834]
    assert O.prng_uniform(12345, 77, 3).tolist() == [0.5454111099243164, -0.27885448932647705, -0.36689019203186035]
