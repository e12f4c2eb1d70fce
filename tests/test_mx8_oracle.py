"""CPU checks of the oracle's OCP MX-fp8 restatement (BASELINE config 5), the rule libwmx's MX-fp8 encoder follows
(wmx_common.h mx8_exp / v_cvt_pk_fp8_f32; tools/mx8_check.hip pins the hardware side on the GPU box).

No reference fixture exists for fp8 (faster-whisper / CTranslate2 have no fp8 mode): parity unpinned against the
reference; pinned instead to the OCP e4m3 code table enumerated here and to the hardware primitive check."""
import numpy as np

from oracle import whisper_np as O


def _codes():
    vals = []
    for b in range(256):
        s, e, m = b >> 7, (b >> 3) & 15, b & 7
        if e == 15 and m == 7:
            continue  # NaN
        v = (m / 8) * 2.0 ** -6 if e == 0 else (1 + m / 8) * 2.0 ** (e - 7)
        vals.append(-v if s else v)
    return np.array(sorted(set(vals)), np.float64)


def test_e4m3_round_is_nearest_even_over_the_code_table():
    codes = _codes()
    assert codes.max() == 448.0 and len(codes) == 253  # +-0 collapse
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.standard_normal(100000) * 40, rng.uniform(-448, 448, 100000),
                        rng.uniform(-2 ** -5, 2 ** -5, 50000), (codes[:-1] + codes[1:]) / 2]).astype(np.float32)
    x = np.clip(x, -448, 448)
    r = O.e4m3_round(x).astype(np.float64)
    assert np.isin(r, codes).all()
    i = np.clip(np.searchsorted(codes, x), 1, len(codes) - 1)
    lo, hi = codes[i - 1], codes[i]
    best = np.minimum(np.abs(x - lo), np.abs(x - hi))
    np.testing.assert_array_equal(np.abs(r - x) <= best, True)
    # exact ties (midpoints) go to the even mantissa
    mids = ((codes[:-1] + codes[1:]) / 2).astype(np.float32)
    rm = O.e4m3_round(mids)
    for v in rm[np.abs(rm) >= 2 ** -6]:
        m, k = np.frexp(abs(float(v)))
        assert int(round((m * 2 - 1) * 8)) % 2 == 0, v


def test_mx8_block_exponent_is_the_smallest_power_of_two():
    rng = np.random.default_rng(4)
    amax = np.abs(rng.standard_normal(20000) * 10 ** rng.uniform(-3, 3, 20000)).astype(np.float32)
    e = O.mx8_exp(amax).astype(np.float64)
    assert np.all(amax / 2.0 ** e <= 448.0)
    assert np.all(amax / 2.0 ** (e - 1) > 448.0)
    np.testing.assert_array_equal(O.mx8_exp(np.array([448.0, 449.0, 1.0], np.float32)), [0, 1, -8])


def test_mx8_quantize_round_trip_properties():
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((16, 256)) * rng.uniform(0.01, 100, (16, 1))).astype(np.float32)
    q = O.mx8_quantize(x)
    np.testing.assert_array_equal(O.mx8_quantize(q), q)  # idempotent
    b = x.reshape(16, 8, 32)
    rel = np.abs(q.reshape(16, 8, 32) - b) / np.abs(b).max(-1, keepdims=True)
    assert rel.max() <= 2.0 ** -4  # half an e4m3 ulp at the top binade, relative to the block max
    assert np.linalg.norm(q - x) / np.linalg.norm(x) < 0.05


def test_fp8_decode_rules():
    """The fp8 decode's oracle rules (oracle/whisper_np.py w8_rows / kv8_images / fp8_decoder_weights): one MX
    power-of-two scale per weight row (per (window, head) image for K / V), every value an e4m3 code times its scale,
    no saturation (row max <= 448 x scale), idempotent; the embedding lookup keeps the 16-bit table while the logits
    projection is quantized; the cross k / v projection weights themselves stay 16-bit (their OUTPUT is quantized)."""
    rng = np.random.default_rng(0)
    w = (rng.standard_normal((64, 1280)) * 0.03).astype(np.float32)
    q = O.w8_rows(w)
    np.testing.assert_array_equal(O.w8_rows(q), q)
    sc = np.ldexp(1.0, O.mx8_exp(np.abs(w).max(-1)))[:, None]
    np.testing.assert_array_equal(O.e4m3_round((q / sc).astype(np.float32)), (q / sc).astype(np.float32))
    assert np.all(np.abs(q / sc) <= 448)
    rel = np.linalg.norm(q - w) / np.linalg.norm(w)
    assert 0.01 < rel < 0.04, rel  # e4m3: 3 mantissa bits
    k = (rng.standard_normal((1500, 256)) * 2.0).astype(np.float32)
    k8 = O.kv8_images(k, 4)
    for h in range(4):
        blk = k8[:, 64 * h: 64 * h + 64]
        s = np.ldexp(1.0, O.mx8_exp(np.abs(O.round_bf16(k[:, 64 * h: 64 * h + 64])).max()))
        np.testing.assert_array_equal(O.e4m3_round((blk / s).astype(np.float32)), (blk / s).astype(np.float32))
    d = O.DIMS["micro"]
    W = O.make_weights(d, 3, "bf16")
    V = O.fp8_decoder_weights(W, d)
    assert V["decoder.kv8"] is True
    np.testing.assert_array_equal(V["decoder.embed_tokens.weight"], W["decoder.embed_tokens.weight"])
    np.testing.assert_array_equal(V["decoder.proj_out.weight"], O.w8_rows(W["decoder.embed_tokens.weight"]))
    for n in ("encoder_attn.k_proj", "encoder_attn.v_proj"):
        np.testing.assert_array_equal(V[f"decoder.layers.0.{n}.weight"], W[f"decoder.layers.0.{n}.weight"])
    for n in O.FP8_DEC_LINEARS:
        key = f"decoder.layers.1.{n}.weight"
        assert not np.array_equal(V[key], W[key]), key
    np.testing.assert_array_equal(V["encoder.layers.0.fc1.weight"], W["encoder.layers.0.fc1.weight"])
