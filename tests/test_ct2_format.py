"""CTranslate2 model.bin ingestion (wmx.ct2; the reference loads CT2 directories, 一键.py:1115).
CTranslate2 is not installed here, so parity with its own files is unpinned: the format (binary version 6, the Whisper
spec's fused variable names, int8 per-row scales) is restated and checked by round trips through the writer; the GPU
test (tests/test_gpu_checkpoint.py) loads such a directory into a model and transcribes."""
import struct

import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import ct2


def _hf(d, seed=1):
    rng = np.random.default_rng(seed)
    sd = {name: rng.standard_normal(shape).astype(np.float32) * 0.05 for name, shape, _, _ in O.tensor_specs(d)}
    sd["encoder.embed_positions.weight"] = rng.standard_normal((1500, d.n_audio_state)).astype(np.float32)
    return sd


def _dims(d):
    return dict(n_audio_layer=d.n_audio_layer, n_text_layer=d.n_text_layer)


@pytest.mark.parametrize("q,tol", [("float32", 0.0), ("float16", 1e-3), ("bfloat16", 8e-3), ("int8", 1.2e-2)])
def test_roundtrip_through_model_bin(tmp_path, q, tol):
    d = O.DIMS["micro"]
    sd = _hf(d)
    v, al = ct2.hf_to_ct2(sd, _dims(d), q)
    p = str(tmp_path / "model.bin")
    ct2.write_model_bin(p, v, al)
    spec, rev, back, aliases = ct2.read_model_bin(p)
    assert spec == "WhisperSpec" and aliases == {"decoder/projection/weight": "decoder/embeddings/weight"}
    dims, hf = ct2.ct2_to_hf(back)
    assert dims["n_audio_state"] == d.n_audio_state and dims["n_text_layer"] == d.n_text_layer
    assert dims["n_mels"] == d.n_mels and dims["n_vocab"] == d.n_vocab and dims["n_audio_head"] * 64 == d.n_audio_state
    for k, ref in sd.items():
        if k.endswith("k_proj.bias"):
            continue
        got = hf[k]
        assert got.shape == ref.shape, k
        err = float(np.max(np.abs(got - ref)) / max(1e-6, float(np.max(np.abs(ref)))))
        lin = k.endswith(".weight") and ("proj" in k or "fc" in k or "embed_tokens" in k)
        assert err <= (tol if lin else 0.0), (k, err)
    assert not any(k.endswith("k_proj.bias") for k in hf)  # Whisper keys have no bias (zeros in the fused CT2 bias)


def test_format_layout(tmp_path):
    """Byte layout of the header and of one variable record, as CTranslate2 writes it."""
    p = str(tmp_path / "model.bin")
    ct2.write_model_bin(p, {"a/b": np.arange(6, dtype=np.float32).reshape(2, 3), "n": np.array(7, np.int16)})
    raw = open(p, "rb").read()
    assert struct.unpack("<I", raw[:4])[0] == 6
    n = struct.unpack("<H", raw[4:6])[0]
    assert raw[6:6 + n] == b"WhisperSpec\0"
    off = 6 + n + 4
    assert struct.unpack("<I", raw[off:off + 4])[0] == 2
    off += 4
    assert struct.unpack("<H", raw[off:off + 2])[0] == 4 and raw[off + 2:off + 6] == b"a/b\0"
    off += 6
    assert raw[off] == 2 and struct.unpack("<2I", raw[off + 1:off + 9]) == (2, 3) and raw[off + 9] == 0
    assert struct.unpack("<I", raw[off + 10:off + 14])[0] == 24
    _, _, v, _ = ct2.read_model_bin(p)
    assert v["n"].shape == () and int(v["n"]) == 7 and v["a/b"][1, 2] == 5.0


def test_rejects_unknown_versions(tmp_path):
    p = tmp_path / "model.bin"
    p.write_bytes(struct.pack("<I", 99))
    with pytest.raises(ValueError):
        ct2.read_model_bin(str(p))


@pytest.mark.parametrize("d,mels,dec,name", [(384, 80, 4, "tiny"), (512, 80, 6, "base"), (1280, 128, 32, "large-v3"),
                                             (1280, 128, 4, "large-v3-turbo"), (1280, 80, 32, "large-v2")])
def test_model_size_inferred_from_a_ct2_dir(tmp_path, d, mels, dec, name):
    """WhisperModel(model_size_or_path=<CT2 dir>) picks the architecture from the tensor shapes (CT2's config.json
    has no d_model)."""
    from wmx.transcribe import _infer_name
    v = {"encoder/conv1/weight": np.zeros((d, mels, 3), np.float16),
         "encoder/position_encodings/encodings": np.zeros((1500, 1), np.float16),
         "decoder/position_encodings/encodings": np.zeros((448, 1), np.float16),
         "decoder/embeddings/weight": np.zeros((10, d), np.float16),
         "encoder/layer_0/ffn/layer_norm/gamma": np.zeros(1, np.float32)}
    for i in range(dec):
        v[f"decoder/layer_{i}/ffn/layer_norm/gamma"] = np.zeros(1, np.float32)
    ct2.write_model_bin(str(tmp_path / "model.bin"), v)
    (tmp_path / "config.json").write_text('{"alignment_heads": [[2, 2]], "suppress_ids": [1, 2]}')
    assert _infer_name(str(tmp_path)) == name


def test_checkpoint_alignment_heads(tmp_path):
    from wmx.transcribe import _checkpoint_alignment_heads
    assert _checkpoint_alignment_heads(None) is None and _checkpoint_alignment_heads(str(tmp_path)) is None
    (tmp_path / "config.json").write_text('{"alignment_heads": [[2, 3], [3, 0]], "lang_ids": [1]}')
    assert _checkpoint_alignment_heads(str(tmp_path)) == [(2, 3), (3, 0)]
    (tmp_path / "config.json").write_text('{"d_model": 384}')
    (tmp_path / "generation_config.json").write_text('{"alignment_heads": [[1, 1]]}')
    assert _checkpoint_alignment_heads(str(tmp_path)) == [(1, 1)]


def test_aliased_layer_variables_resolve(tmp_path):
    """CTranslate2's converter stores a variable equal to an earlier one as an alias: a LayerNorm beta and
    a bias deduplicated that way, plus an alias chain, load as their targets' values."""
    d = O.DIMS["micro"]
    sd = _hf(d)
    sd["decoder.layers.1.final_layer_norm.bias"] = sd["decoder.layers.0.final_layer_norm.bias"].copy()
    sd["encoder.layers.1.fc2.bias"] = sd["encoder.layers.0.fc2.bias"].copy()
    v, al = ct2.hf_to_ct2(sd, _dims(d), "float32")
    al = dict(al)
    al["decoder/layer_1/ffn/layer_norm/beta"] = "decoder/layer_0/ffn/layer_norm/beta"
    al["encoder/layer_1/ffn/linear_1/bias"] = "encoder/layer_0/ffn/linear_1/bias"
    del v["decoder/layer_1/ffn/layer_norm/beta"], v["encoder/layer_1/ffn/linear_1/bias"]
    p = tmp_path / "model.bin"
    ct2.write_model_bin(str(p), v, al)
    dims, hf = ct2.load_ct2_dir(str(tmp_path))
    np.testing.assert_array_equal(hf["decoder.layers.1.final_layer_norm.bias"], sd["decoder.layers.0.final_layer_norm.bias"])
    np.testing.assert_array_equal(hf["encoder.layers.1.fc2.bias"], sd["encoder.layers.0.fc2.bias"])
    chained = ct2.resolve_aliases({"x": np.ones(2)}, {"a": "b", "b": "x"})
    np.testing.assert_array_equal(chained["a"], np.ones(2))
    with pytest.raises(KeyError):
        ct2.resolve_aliases({}, {"a": "missing"})


def test_int8_grid_rule_and_exact_recovery():
    """The CTranslate2 int8 rule (oracle.int8_rows: scale = 127 / max|row|, 1 for a zero row, q = rint(w scale); the
    formula of the CT2 export restatement wmx.ct2.hf_to_ct2), and a CT2 int8 checkpoint's q is recovered EXACTLY from its
    dequantized weights rounded to 16 bits with the checkpoint's own scales -- the property the int8 model's device
    quantization relies on (|q| <= 127 and a 16-bit rounding <= 2^-9 relative keep |w scale - q| < 1/2)."""
    import torch
    from oracle import whisper_np as O
    rng = np.random.default_rng(4)
    w = (rng.standard_normal((256, 640)) * 0.05).astype(np.float32)
    w[7] = 0.0  # an all-zero row: scale 1, q 0
    q, s = O.int8_rows(w)
    assert q.dtype == np.int8 and np.abs(q).max() == 127 and s[7] == 1.0 and not q[7].any()
    for dt in (torch.bfloat16, torch.float16):
        w16 = torch.from_numpy(q.astype(np.float32) / s[:, None]).to(dt).float().numpy()
        q2, s2 = O.int8_rows(w16, s)
        np.testing.assert_array_equal(q2, q)
        np.testing.assert_array_equal(s2, s)


def test_ct2_to_hf_keeps_int8_row_scales():
    """An int8 CT2 export read back: ct2_to_hf returns the dequantized weights and, for the weights an int8 model keeps
    on the int8 grid (decoder projections, the fused q | k | v split per projection, the token embedding), the
    checkpoint's row scales by HF name -- never for the encoder or the cross-attention K / V projection."""
    from oracle import whisper_np as O
    d = O.DIMS["micro"]
    W = O.make_weights(d, 3, "bf16")
    sd = {k: v for k, v in W.items() if k != "encoder.embed_positions.weight"}
    sd["encoder.embed_positions.weight"] = W["encoder.embed_positions.weight"]
    v, al = ct2.hf_to_ct2(sd, dict(n_audio_layer=d.n_audio_layer, n_text_layer=d.n_text_layer), "int8")
    scales = {}
    dims, out = ct2.ct2_to_hf(ct2.resolve_aliases(v, al), scales)
    dt = d.n_text_state
    want = {"decoder.embed_tokens.weight"}
    for i in range(d.n_text_layer):
        for n in O.FP8_DEC_LINEARS:
            want.add(f"decoder.layers.{i}.{n}.weight")
    assert set(scales) == want
    s_qkv = v["decoder/layer_0/self_attention/linear_0/weight_scale"]
    np.testing.assert_array_equal(scales["decoder.layers.0.self_attn.k_proj.weight"], s_qkv[dt:2 * dt])
    q_fc1 = v["decoder/layer_0/ffn/linear_0/weight"]
    np.testing.assert_array_equal(O.int8_rows(out["decoder.layers.0.fc1.weight"],
                                              scales["decoder.layers.0.fc1.weight"])[0], q_fc1)
