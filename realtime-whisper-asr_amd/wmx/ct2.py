"""CTranslate2 `model.bin` ingestion: the reference app loads faster-whisper models from a
CT2 directory (`models_fast/`, 一键实时识别麦克风.py:1115), so a user switching engines has CT2 files, not HF
safetensors.  This module restates the CT2 model format (CTranslate2 4.x `ModelSpec._serialize`, binary version
6 -- the engine is not installed here, so parity is unpinned: it is checked by writing and reading back files of
this format, `write_model_bin`, and end to end on the GPU against the synthetic weights):

    uint32 binary_version (3..6) | string spec_name | uint32 spec_revision | uint32 n_variables
    n x { string name | uint8 rank | uint32 dims[rank] | uint8 dtype | uint32 n_bytes | bytes }
    uint32 n_aliases | n x { string alias | string target }
    string = uint16 length (with the NUL) + bytes + NUL; dtype: 0 f32, 1 int8, 2 int16, 3 int32, 4 f16, 5 bf16

and the CT2 Whisper spec's variable names (the transformers converter's layout): fused self-attention q|k|v
(`self_attention/linear_0`, k without bias -> zeros), fused cross-attention k|v (`attention/linear_1`), int8
weights with a per-row `weight_scale` (w = q / scale).  `ct2_to_hf` maps them onto the HF names
`wmx_model_set_tensor` takes.
"""
from __future__ import annotations

import os
import re
import struct

import numpy as np

_DT = {0: (np.float32, 4), 1: (np.int8, 1), 2: (np.int16, 2), 3: (np.int32, 4), 4: (np.float16, 2), 5: (None, 2)}


def _read_string(f):
    (n,) = struct.unpack("<H", f.read(2))
    raw = f.read(n)
    return raw[:-1].decode() if raw.endswith(b"\0") else raw.decode()


def read_model_bin(path: str):
    """-> (spec_name, revision, {name: array (f32 / int8 / int16 / int32; bf16 and f16 widened to f32)},
    {alias: target})."""
    with open(path, "rb") as f:
        (version,) = struct.unpack("<I", f.read(4))
        if not 3 <= version <= 6:
            raise ValueError(f"{path}: CT2 binary version {version} is not supported (3..6)")
        spec = _read_string(f)
        (revision,) = struct.unpack("<I", f.read(4))
        (nvar,) = struct.unpack("<I", f.read(4))
        out = {}
        for _ in range(nvar):
            name = _read_string(f)
            (rank,) = struct.unpack("<B", f.read(1))
            shape = struct.unpack(f"<{rank}I", f.read(4 * rank)) if rank else ()
            (dt,) = struct.unpack("<B", f.read(1))
            (nbytes,) = struct.unpack("<I", f.read(4))
            buf = f.read(nbytes)
            if dt not in _DT:
                raise ValueError(f"{path}: variable {name}: unknown CT2 dtype {dt}")
            npdt, size = _DT[dt]
            if nbytes != int(np.prod(shape, dtype=np.int64)) * size:
                raise ValueError(f"{path}: variable {name}: {nbytes} bytes for shape {shape}")
            if dt == 5:  # bf16: the high half of an f32
                a = (np.frombuffer(buf, np.uint16).astype(np.uint32) << 16).view(np.float32)
            else:
                a = np.frombuffer(buf, npdt)
                if dt == 4:
                    a = a.astype(np.float32)
            out[name] = a.reshape(shape)
        aliases = {}
        tail = f.read(4)
        if tail:
            (nal,) = struct.unpack("<I", tail)
            for _ in range(nal):
                a = _read_string(f)
                aliases[a] = _read_string(f)
    return spec, revision, out, aliases


def _write_string(f, s):
    b = s.encode()
    f.write(struct.pack("<H", len(b) + 1))
    f.write(b + b"\0")


def write_model_bin(path: str, variables: dict, aliases: dict | None = None, spec: str = "WhisperSpec",
                    revision: int = 3):
    """The same format (binary version 6): arrays of float32 / int8 / int16 / int32 / float16; a variable given as
    ('bf16', f32 array) is stored as bfloat16 (round to nearest even)."""
    code = {np.dtype(np.float32): 0, np.dtype(np.int8): 1, np.dtype(np.int16): 2, np.dtype(np.int32): 3,
            np.dtype(np.float16): 4}
    with open(path, "wb") as f:
        f.write(struct.pack("<I", 6))
        _write_string(f, spec)
        f.write(struct.pack("<I", revision))
        f.write(struct.pack("<I", len(variables)))
        for name, v in variables.items():
            if isinstance(v, tuple) and v[0] == "bf16":
                x = np.ascontiguousarray(v[1], np.float32)
                u = x.view(np.uint32)
                raw = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16).tobytes()
                dt, shape = 5, x.shape
            else:
                x = np.asarray(v)  # (np.ascontiguousarray would turn a 0-d scalar into shape (1,))
                dt, shape, raw = code[x.dtype], x.shape, x.tobytes(order="C")
            _write_string(f, name)
            f.write(struct.pack("<B", len(shape)))
            if shape:
                f.write(struct.pack(f"<{len(shape)}I", *shape))
            f.write(struct.pack("<B", dt))
            f.write(struct.pack("<I", len(raw)))
            f.write(raw)
        aliases = aliases or {}
        f.write(struct.pack("<I", len(aliases)))
        for a, t in aliases.items():
            _write_string(f, a)
            _write_string(f, t)


def _weight(v, prefix):
    """A CT2 linear's weight as f32: int8 rows dequantised by their per-row scale (w = q / scale)."""
    w = v[prefix + "/weight"]
    if w.dtype == np.int8 or w.dtype == np.int16:
        s = np.asarray(v[prefix + "/weight_scale"], np.float32).reshape(-1, 1)
        return w.astype(np.float32) / s
    return np.asarray(w, np.float32)


def _bias(v, prefix, n):
    b = v.get(prefix + "/bias")
    return np.zeros(n, np.float32) if b is None else np.asarray(b, np.float32)


def ct2_dims(v):
    """ModelDimensions from the variable shapes (head dim 64, as every Whisper size)."""
    d, M = v["encoder/conv1/weight"].shape[:2]
    enc_l = len({int(m.group(1)) for k in v for m in [re.match(r"encoder/layer_(\d+)/", k)] if m})
    dec_l = len({int(m.group(1)) for k in v for m in [re.match(r"decoder/layer_(\d+)/", k)] if m})
    V, dt = v["decoder/embeddings/weight"].shape
    return dict(n_mels=int(M), n_vocab=int(V), n_audio_ctx=int(v["encoder/position_encodings/encodings"].shape[0]),
                n_audio_state=int(d), n_audio_head=int(d) // 64, n_audio_layer=enc_l,
                n_text_ctx=int(v["decoder/position_encodings/encodings"].shape[0]), n_text_state=int(dt),
                n_text_head=int(dt) // 64, n_text_layer=dec_l)


# the weights an int8 model (WMX_DTYPE_I8) keeps on CTranslate2's int8 grid: every decoder projection the decode step
# streams and the token embedding (the logits projection); the encoder and the cross-attention K / V projection run
# on the dequantized 16-bit weights
_I8_KEPT = re.compile(r"decoder\.(embed_tokens|layers\.\d+\.(self_attn\.(q|k|v|out)_proj|encoder_attn\.(q|out)_proj|fc1|fc2))"
                      r"\.weight$")


def ct2_to_hf(v, row_scales: dict | None = None):
    """CT2 Whisper variables -> the HF state dict (f32, without the "model." prefix) wmx_model_set_tensor takes.
    row_scales (optional dict, filled): the CT2 int8 weight_scale rows of the weights an int8 model keeps on the int8
    grid, by HF weight name (wmx_model_set_row_scales), so that model's q = rint(w * scale) is the checkpoint's q."""
    dims = ct2_dims(v)
    out = {}

    def keep_scale(src, dst, r0=None, r1=None):
        if row_scales is None or not _I8_KEPT.match(dst) or src + "/weight_scale" not in v:
            return
        if v[src + "/weight"].dtype != np.int8:
            return
        sc = np.asarray(v[src + "/weight_scale"], np.float32).reshape(-1)
        row_scales[dst] = sc if r0 is None else sc[r0:r1]

    def ln(src, dst):
        out[dst + ".weight"] = np.asarray(v[src + "/gamma"], np.float32)
        out[dst + ".bias"] = np.asarray(v[src + "/beta"], np.float32)

    def lin(src, dst, bias=True):
        w = _weight(v, src)
        out[dst + ".weight"] = w
        keep_scale(src, dst + ".weight")
        if bias:
            out[dst + ".bias"] = _bias(v, src, w.shape[0])

    def split(src, dsts, d):
        w = _weight(v, src)
        b = _bias(v, src, w.shape[0])
        for j, (dst, has_bias) in enumerate(dsts):
            out[dst + ".weight"] = w[j * d:(j + 1) * d]
            keep_scale(src, dst + ".weight", j * d, (j + 1) * d)
            if has_bias:
                out[dst + ".bias"] = b[j * d:(j + 1) * d]

    for c in ("conv1", "conv2"):
        w = v[f"encoder/{c}/weight"]
        if w.dtype == np.int8:  # quantized per output channel like a linear weight
            w = (w.reshape(w.shape[0], -1).astype(np.float32)
                 / np.asarray(v[f"encoder/{c}/weight_scale"], np.float32).reshape(-1, 1)).reshape(w.shape)
        out[f"encoder.{c}.weight"] = np.asarray(w, np.float32)
        out[f"encoder.{c}.bias"] = np.asarray(v[f"encoder/{c}/bias"], np.float32)
    out["encoder.embed_positions.weight"] = np.asarray(v["encoder/position_encodings/encodings"], np.float32)
    ln("encoder/layer_norm", "encoder.layer_norm")
    da, dt = dims["n_audio_state"], dims["n_text_state"]
    for i in range(dims["n_audio_layer"]):
        s, h = f"encoder/layer_{i}", f"encoder.layers.{i}"
        ln(s + "/self_attention/layer_norm", h + ".self_attn_layer_norm")
        split(s + "/self_attention/linear_0",
              [(h + ".self_attn.q_proj", True), (h + ".self_attn.k_proj", False), (h + ".self_attn.v_proj", True)], da)
        lin(s + "/self_attention/linear_1", h + ".self_attn.out_proj")
        ln(s + "/ffn/layer_norm", h + ".final_layer_norm")
        lin(s + "/ffn/linear_0", h + ".fc1")
        lin(s + "/ffn/linear_1", h + ".fc2")
    out["decoder.embed_tokens.weight"] = _weight(v, "decoder/embeddings") if "decoder/embeddings/weight_scale" in v \
        else np.asarray(v["decoder/embeddings/weight"], np.float32)
    keep_scale("decoder/embeddings", "decoder.embed_tokens.weight")
    out["decoder.embed_positions.weight"] = np.asarray(v["decoder/position_encodings/encodings"], np.float32)
    ln("decoder/layer_norm", "decoder.layer_norm")
    for i in range(dims["n_text_layer"]):
        s, h = f"decoder/layer_{i}", f"decoder.layers.{i}"
        ln(s + "/self_attention/layer_norm", h + ".self_attn_layer_norm")
        split(s + "/self_attention/linear_0",
              [(h + ".self_attn.q_proj", True), (h + ".self_attn.k_proj", False), (h + ".self_attn.v_proj", True)], dt)
        lin(s + "/self_attention/linear_1", h + ".self_attn.out_proj")
        ln(s + "/attention/layer_norm", h + ".encoder_attn_layer_norm")
        lin(s + "/attention/linear_0", h + ".encoder_attn.q_proj")
        split(s + "/attention/linear_1", [(h + ".encoder_attn.k_proj", False), (h + ".encoder_attn.v_proj", True)], dt)
        lin(s + "/attention/linear_2", h + ".encoder_attn.out_proj")
        ln(s + "/ffn/layer_norm", h + ".final_layer_norm")
        lin(s + "/ffn/linear_0", h + ".fc1")
        lin(s + "/ffn/linear_1", h + ".fc2")
    return dims, out


def hf_to_ct2(sd, dims, quantize: str = "float32"):
    """The inverse map (an export / test fixture): HF names -> CT2 Whisper variables, quantize in
    {"float32", "float16", "bfloat16", "int8"} (int8: linear weights per-row, scale = 127 / max|row|, as CT2)."""
    v = {}

    def W(name, w):
        w = np.asarray(w, np.float32)
        if quantize == "int8":
            amax = np.abs(w).max(axis=1)
            amax[amax == 0] = 127.0
            scale = (127.0 / amax).astype(np.float32)
            v[name + "/weight"] = np.rint(w * scale[:, None]).astype(np.int8)
            v[name + "/weight_scale"] = scale
        elif quantize == "float16":
            v[name + "/weight"] = w.astype(np.float16)
        elif quantize == "bfloat16":
            v[name + "/weight"] = ("bf16", w)
        else:
            v[name + "/weight"] = w

    def f32(name, a):
        v[name] = np.asarray(a, np.float32)

    def ln(dst, src):
        f32(dst + "/gamma", sd[src + ".weight"])
        f32(dst + "/beta", sd[src + ".bias"])

    def fused(dst, srcs):
        W(dst, np.concatenate([sd[s + ".weight"] for s in srcs]))
        f32(dst + "/bias", np.concatenate([sd.get(s + ".bias", np.zeros(np.asarray(sd[s + ".weight"]).shape[0]))
                                           for s in srcs]))

    def lin(dst, src):
        W(dst, sd[src + ".weight"])
        f32(dst + "/bias", sd[src + ".bias"])

    for c in ("conv1", "conv2"):
        f32(f"encoder/{c}/weight", sd[f"encoder.{c}.weight"])
        f32(f"encoder/{c}/bias", sd[f"encoder.{c}.bias"])
    f32("encoder/position_encodings/encodings", sd["encoder.embed_positions.weight"])
    ln("encoder/layer_norm", "encoder.layer_norm")
    for i in range(dims["n_audio_layer"]):
        s, h = f"encoder/layer_{i}", f"encoder.layers.{i}"
        ln(s + "/self_attention/layer_norm", h + ".self_attn_layer_norm")
        fused(s + "/self_attention/linear_0", [h + ".self_attn.q_proj", h + ".self_attn.k_proj", h + ".self_attn.v_proj"])
        lin(s + "/self_attention/linear_1", h + ".self_attn.out_proj")
        ln(s + "/ffn/layer_norm", h + ".final_layer_norm")
        lin(s + "/ffn/linear_0", h + ".fc1")
        lin(s + "/ffn/linear_1", h + ".fc2")
    W("decoder/embeddings", sd["decoder.embed_tokens.weight"])
    f32("decoder/position_encodings/encodings", sd["decoder.embed_positions.weight"])
    ln("decoder/layer_norm", "decoder.layer_norm")
    for i in range(dims["n_text_layer"]):
        s, h = f"decoder/layer_{i}", f"decoder.layers.{i}"
        ln(s + "/self_attention/layer_norm", h + ".self_attn_layer_norm")
        fused(s + "/self_attention/linear_0", [h + ".self_attn.q_proj", h + ".self_attn.k_proj", h + ".self_attn.v_proj"])
        lin(s + "/self_attention/linear_1", h + ".self_attn.out_proj")
        ln(s + "/attention/layer_norm", h + ".encoder_attn_layer_norm")
        lin(s + "/attention/linear_0", h + ".encoder_attn.q_proj")
        fused(s + "/attention/linear_1", [h + ".encoder_attn.k_proj", h + ".encoder_attn.v_proj"])
        lin(s + "/attention/linear_2", h + ".encoder_attn.out_proj")
        ln(s + "/ffn/layer_norm", h + ".final_layer_norm")
        lin(s + "/ffn/linear_0", h + ".fc1")
        lin(s + "/ffn/linear_1", h + ".fc2")
    return v, {"decoder/projection/weight": "decoder/embeddings/weight"}


def resolve_aliases(v: dict, aliases: dict) -> dict:
    """The variable dict with every alias bound to its target's array.  CTranslate2's converter replaces ANY variable
    that is element-wise equal to an earlier one (in name order) with an alias, not only the tied output projection:
    a fine-tuned or distilled model can store e.g. identical LayerNorm or bias vectors once.  Chains resolve."""
    out = dict(v)
    for a in aliases:
        t, seen = aliases[a], {a}
        while t not in out and t in aliases and t not in seen:
            seen.add(t)
            t = aliases[t]
        if t not in out:
            raise KeyError(f"CT2 alias {a!r} -> {aliases[a]!r}: target not in the model")
        out.setdefault(a, out[t])
    return out


def load_ct2_dir(model_dir: str, row_scales: dict | None = None):
    """(dims, HF state dict) of a CT2 Whisper model directory (model.bin), aliases resolved; row_scales as ct2_to_hf."""
    _, _, v, aliases = read_model_bin(os.path.join(model_dir, "model.bin"))
    return ct2_to_hf(resolve_aliases(v, aliases), row_scales)
