"""numpy restatement of the streaming-Whisper hot path (TEST INFRASTRUCTURE ONLY).

See ``oracle/__init__.py`` for scope and pinning.  Every function cites what it
restates.  Arithmetic is float32 (log-mel float64), i.e. the exact-math
reference the bf16/fp16 HIP path is compared against.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
from scipy.special import erf

SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160
N_SAMPLES = 480000          # 30 s window
N_FRAMES = 3000             # mel frames per window
N_AUDIO_CTX = 1500          # encoder positions
N_TEXT_CTX = 448


# ----------------------------------------------------------------------------------------------
# model dimensions (openai-whisper ModelDimensions; CT2 converted models carry the same numbers)
# ----------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Dims:
    n_mels: int
    n_vocab: int
    n_audio_state: int
    n_audio_head: int
    n_audio_layer: int
    n_text_state: int
    n_text_head: int
    n_text_layer: int
    n_audio_ctx: int = N_AUDIO_CTX
    n_text_ctx: int = N_TEXT_CTX


DIMS = {
    "tiny": Dims(80, 51865, 384, 6, 4, 384, 6, 4),
    "base": Dims(80, 51865, 512, 8, 6, 512, 8, 6),
    "small": Dims(80, 51865, 768, 12, 12, 768, 12, 12),
    "medium": Dims(80, 51865, 1024, 16, 24, 1024, 16, 24),
    "large-v3": Dims(128, 51866, 1280, 20, 32, 1280, 20, 32),
    "large-v3-turbo": Dims(128, 51866, 1280, 20, 32, 1280, 20, 4),
    # a deliberately small configuration for fast parity tests (not a released model)
    "micro": Dims(80, 51865, 128, 2, 2, 128, 2, 2),
}


# ----------------------------------------------------------------------------------------------
# special tokens (openai-whisper tokenizer.py; faster-whisper Tokenizer wraps the same ids)
# ----------------------------------------------------------------------------------------------
LANGUAGES = [
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it",
    "id", "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur",
    "hr", "bg", "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn",
    "et", "mk", "br", "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si",
    "km", "sn", "yo", "so", "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo",
    "ht", "ps", "tk", "nn", "mt", "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha",
    "ba", "jw", "su", "yue",
]


@dataclass(frozen=True)
class Special:
    eot: int
    sot: int
    lang0: int
    n_langs: int
    translate: int
    transcribe: int
    sot_lm: int
    sot_prev: int
    no_speech: int
    no_timestamps: int
    timestamp_begin: int
    blank: int = 220  # " " in the GPT-2 byte-level BPE


def special_tokens(n_vocab: int) -> Special:
    """openai-whisper tokenizer: large-v3 (51866) adds "yue" and shifts every id after the languages by one."""
    n_langs = 100 if n_vocab >= 51866 else 99
    base = 50258 + 1 + n_langs  # first id after the language tokens
    return Special(eot=50257, sot=50258, lang0=50259, n_langs=n_langs, translate=base,
                   transcribe=base + 1, sot_lm=base + 2, sot_prev=base + 3, no_speech=base + 4,
                   no_timestamps=base + 5, timestamp_begin=base + 6)


# ----------------------------------------------------------------------------------------------
# build-owned deterministic weight PRNG (same algorithm as csrc/wmx_weights.hip)
# ----------------------------------------------------------------------------------------------
_M64 = (1 << 64) - 1
_G1 = 0x9E3779B97F4A7C15
_G2 = 0xBF58476D1CE4E5B9
_G3 = 0x94D049BB133111EB


def prng_uniform(seed: int, tid: int, n: int) -> np.ndarray:
    """u in [-1, 1) for element indices 0..n-1 of tensor `tid`: splitmix64 of a counter, top 24 bits."""
    key = np.uint64((seed * _G1 + tid * _G2) & _M64)
    z = np.arange(n, dtype=np.uint64) + key
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_G2)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_G3)
        z = z ^ (z >> np.uint64(31))
    k = (z >> np.uint64(40)).astype(np.float32)  # < 2^24, exact
    return k * np.float32(2.0 ** -23) - np.float32(1.0)  # exact in fp32


def round_bf16(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) << np.uint64(16)
    return r.astype(np.uint32).view(np.float32)


def round_dtype(x: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "bf16":
        return round_bf16(x)
    if dtype == "f16":
        return x.astype(np.float16).astype(np.float32)
    return x.astype(np.float32)


# ----------------------------------------------------------------------------------------------
# OCP MX-fp8 (BASELINE config 5: the encoder projections on the CDNA4 MX-fp8 MFMA).  No reference fixture exists
# for this path (faster-whisper/CT2 have no fp8 mode; the reference CPU config is int8): the rule below restates
# the OCP Microscaling spec's fp8 e4m3 element format with one e8m0 scale per 32 consecutive K elements, the
# scale chosen as the smallest power of two that brings the block max within the e4m3 range (no saturation);
# tools/mx8_check.hip pins the hardware conversion (round-to-nearest-even) and the scaled-MFMA lane maps.
# ----------------------------------------------------------------------------------------------
def mx8_exp(amax: np.ndarray) -> np.ndarray:
    """Block exponent e (scale 2^e): amax = m 2^k, m in [0.5, 1) -> e = k - 9 + (m > 0.875), clamped to [-126, 126]
    (the float32 bits of amax, exactly as wmx_common.h mx8_exp)."""
    u = np.ascontiguousarray(amax, dtype=np.float32).view(np.uint32)
    E = ((u >> np.uint32(23)) & np.uint32(255)).astype(np.int32)
    Mt = (u & np.uint32(0x7FFFFF)).astype(np.int32)
    return np.clip(E - 135 + (Mt > 0x600000), -126, 126).astype(np.int32)


def e4m3_round(v: np.ndarray) -> np.ndarray:
    """Nearest-even OCP e4m3 value of float32 v with |v| <= 448 (subnormal step 2^-9, normal step 2^(E-3))."""
    v = np.asarray(v, dtype=np.float32)
    a = np.abs(v).astype(np.float64)
    m, k = np.frexp(np.maximum(a, 2.0 ** -6))  # a = m 2^k, m in [0.5, 1): binade exponent E = k - 1
    step = np.ldexp(1.0, k - 4)                  # 2^(E-3); at a < 2^-6 the clamp gives the subnormal step 2^-9
    q = np.rint(a / step) * step
    return (np.sign(v) * q).astype(np.float32)


def mx8_quantize(x: np.ndarray, block: int = 32) -> np.ndarray:
    """MX-fp8 round trip along the last axis (blocks of `block`, default 32; the fp8 decode's weights use the whole row,
    w8_rows): the dequantized float32 values the MFMA consumes."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    K = x.shape[-1]
    assert K % block == 0
    b = x.reshape(x.shape[:-1] + (K // block, block))
    e = mx8_exp(np.abs(b).max(-1))[..., None]
    inv = np.ldexp(np.float32(1.0), -e).astype(np.float32)
    q = e4m3_round((b * inv).astype(np.float32))
    return (q.astype(np.float64) * np.ldexp(1.0, e)).astype(np.float32).reshape(x.shape)


# ----------------------------------------------------------------------------------------------
# The fp8 decode of the same model dtype (csrc/wmx_ops.hip w8_quantize_kernel / crosskv_quant_kernel).  Restated
# from this build's own rule -- no reference fixture exists (faster-whisper/CT2 have no fp8 mode; their 8-bit mode,
# int8_float16, quantizes each weight ROW with its own scale, which is the granularity kept here):
#   * every decoder projection (self q/k/v/out, cross q/out, fc1, fc2) and the logits projection (the token
#     embedding, tied) is e4m3 with ONE power-of-two scale per weight row, chosen by the MX rule above over the row;
#     the embedding LOOKUP keeps the 16-bit table;
#   * the cross-attention K / V of every (layer, head) are rounded to the model dtype (the device stores 16-bit images
#     first) and then e4m3 with one power-of-two scale per (layer, window, head) image (1500 keys x 64 dims);
#   * activations, LayerNorms, biases and the self-attention cache are unchanged.
# The device multiplies the fp32 products by the scales outside the MFMA (exact: powers of two).
# ----------------------------------------------------------------------------------------------
FP8_DEC_LINEARS = ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj", "self_attn.out_proj",
                   "encoder_attn.q_proj", "encoder_attn.out_proj", "fc1", "fc2")


def w8_rows(w: np.ndarray) -> np.ndarray:
    """A weight matrix [N][K] through the fp8 decode's rule: e4m3 with one MX power-of-two scale per row."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    return mx8_quantize(w, block=w.shape[-1])


def fp8_decoder_weights(W: dict, d: Dims) -> dict:
    """The weights the fp8 decode computes with: a copy of W whose decoder projections are w8_rows-quantized, with
    the quantized embedding as the separate logits projection ("decoder.proj_out.weight") and the cross-K/V image
    rule switched on ("decoder.kv8", read by DecoderCache)."""
    V = dict(W)
    for i in range(d.n_text_layer):
        for n in FP8_DEC_LINEARS:
            k = f"decoder.layers.{i}.{n}.weight"
            V[k] = w8_rows(W[k])
    V["decoder.proj_out.weight"] = w8_rows(W["decoder.embed_tokens.weight"])
    V["decoder.kv8"] = True
    return V


# ----------------------------------------------------------------------------------------------
# The CTranslate2 int8 grid (the reference's compute_type int8_float16 / int8: 一键实时识别麦克风.py:304,
# asr_components.py:256-261; CTranslate2 4.x int8 quantization, restated -- the engine is not installed here):
#   * every weight row: scale = 127 / max|row| (1 for an all-zero row), q = rint(w * scale) in [-127, 127] (int8);
#     a CT2 int8 checkpoint stores q and scale (w = q / scale);
#   * the device's int8 model keeps every decoder projection (the FP8_DEC_LINEARS) and the logits projection (the tied
#     token embedding) on that grid -- q from its 16-bit weights by the rule, or with a checkpoint's own scales, which
#     recovers the checkpoint's q exactly -- and computes with q / scale (the 16-bit q is exact, the fp32 result is
#     multiplied by 1 / scale); the embedding LOOKUP, the encoder and the cross-attention K / V projection keep the
#     16-bit weights.  (CT2 also quantizes the activations of its int8 GEMMs per row; the device keeps them 16-bit:
#     weight-only int8, parity with CT2's own arithmetic unpinned.)
# ----------------------------------------------------------------------------------------------
def int8_rows(w: np.ndarray, scale=None):
    """(q int8 [N][K], scale f32 [N]) of a weight matrix by CTranslate2's int8 rule; `scale` given (a checkpoint's
    weight_scale) or 127 / max|row| in float32 (the device's arithmetic: f32 division, f32 product, rint half-even)."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    if scale is None:
        amax = np.abs(w).max(axis=1)
        scale = np.where(amax > 0, np.float32(127.0) / np.where(amax > 0, amax, np.float32(1.0)), np.float32(1.0))
    scale = np.asarray(scale, np.float32).reshape(-1)
    q = np.clip(np.rint(w * scale[:, None]), -127, 127).astype(np.int8)
    return q, scale.astype(np.float32)


def int8_decoder_weights(W: dict, d: Dims, scales: dict | None = None) -> dict:
    """The weights the int8 model's decode computes with: a copy of W whose decoder projections are q / scale of
    int8_rows (scales: a CT2 int8 checkpoint's per-row scales by weight name, else CT2's rule on W), and the logits
    projection ("decoder.proj_out.weight") the same of the token embedding; the lookup keeps W's embedding."""
    scales = scales or {}
    V = dict(W)

    def deq(name):
        q, s = int8_rows(W[name], scales.get(name))
        return (q.astype(np.float32) / s[:, None]).astype(np.float32)

    for i in range(d.n_text_layer):
        for n in FP8_DEC_LINEARS:
            k = f"decoder.layers.{i}.{n}.weight"
            V[k] = deq(k)
    V["decoder.proj_out.weight"] = deq("decoder.embed_tokens.weight")
    return V


def kv8_images(x: np.ndarray, n_head: int) -> np.ndarray:
    """Cross K or V [T][d] of one window through the fp8 image rule: bf16, then e4m3 with one MX scale per head."""
    T, dm = x.shape
    xh = round_bf16(x).reshape(T, n_head, dm // n_head).transpose(1, 0, 2).reshape(n_head, -1)
    q = mx8_quantize(xh, block=xh.shape[-1])
    return q.reshape(n_head, T, dm // n_head).transpose(1, 0, 2).reshape(T, dm)


def linear_mx8(x, W, p, bias=True):
    """linear() with both operands MX-fp8-quantized along K (fp32 accumulation of the exact products)."""
    y = mx8_quantize(x).astype(np.float64) @ mx8_quantize(W[p + ".weight"]).astype(np.float64).T
    if bias:
        y = y + W[p + ".bias"]
    return y.astype(np.float32)


def tensor_specs(d: Dims):
    """(name, logical shape, scale, offset) in generation order; tid = index in this list.

    Names follow the HF/openai state-dict naming so a real checkpoint maps 1:1."""
    specs = []
    f32 = lambda v: float(np.float32(v))

    def lin(p, n_out, n_in, bias=True):
        specs.append((p + ".weight", (n_out, n_in), f32(1.0 / math.sqrt(n_in)), 0.0))
        if bias:
            specs.append((p + ".bias", (n_out,), 0.02, 0.0))

    def ln(p, n):
        specs.append((p + ".weight", (n,), 0.1, 1.0))
        specs.append((p + ".bias", (n,), 0.02, 0.0))

    def attn(p, n):
        lin(p + ".q_proj", n, n)
        lin(p + ".k_proj", n, n, bias=False)
        lin(p + ".v_proj", n, n)
        lin(p + ".out_proj", n, n)

    da, dt = d.n_audio_state, d.n_text_state
    specs.append(("encoder.conv1.weight", (da, d.n_mels, 3), f32(1.0 / math.sqrt(3 * d.n_mels)), 0.0))
    specs.append(("encoder.conv1.bias", (da,), 0.02, 0.0))
    specs.append(("encoder.conv2.weight", (da, da, 3), f32(1.0 / math.sqrt(3 * da)), 0.0))
    specs.append(("encoder.conv2.bias", (da,), 0.02, 0.0))
    for i in range(d.n_audio_layer):
        p = f"encoder.layers.{i}"
        ln(p + ".self_attn_layer_norm", da)
        attn(p + ".self_attn", da)
        ln(p + ".final_layer_norm", da)
        lin(p + ".fc1", 4 * da, da)
        lin(p + ".fc2", da, 4 * da)
    ln("encoder.layer_norm", da)
    specs.append(("decoder.embed_tokens.weight", (d.n_vocab, dt), f32(6.0 / math.sqrt(dt)), 0.0))
    specs.append(("decoder.embed_positions.weight", (d.n_text_ctx, dt), 0.05, 0.0))
    for i in range(d.n_text_layer):
        p = f"decoder.layers.{i}"
        ln(p + ".self_attn_layer_norm", dt)
        attn(p + ".self_attn", dt)
        ln(p + ".encoder_attn_layer_norm", dt)
        attn(p + ".encoder_attn", dt)
        ln(p + ".final_layer_norm", dt)
        lin(p + ".fc1", 4 * dt, dt)
        lin(p + ".fc2", dt, 4 * dt)
    ln("decoder.layer_norm", dt)
    return specs


def make_weights(d: Dims, seed: int, dtype: str = "bf16") -> dict:
    """Deterministic synthetic weights, value = u*scale + offset (separately rounded fp32 ops), then
    rounded to the storage dtype.  Returns float32 arrays holding the stored values."""
    W = {}
    for tid, (name, shape, scale, offset) in enumerate(tensor_specs(d)):
        n = int(np.prod(shape))
        u = prng_uniform(seed, tid, n)
        v = u * np.float32(scale)
        if offset != 0.0:
            v = v + np.float32(offset)
        W[name] = round_dtype(v, dtype).reshape(shape)
    W["encoder.embed_positions.weight"] = sinusoids(d.n_audio_ctx, d.n_audio_state)
    return W


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """openai-whisper model.sinusoids (transformers modeling_whisper.py:55), evaluated in float64."""
    inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2, dtype=np.float64))
    t = np.arange(length, dtype=np.float64)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


# ----------------------------------------------------------------------------------------------
# log-mel (faster-whisper 1.2.1 feature_extractor.py FeatureExtractor.__call__, padding=160)
# ----------------------------------------------------------------------------------------------
def mel_filters(n_mels: int, sr: int = SAMPLE_RATE, n_fft: int = N_FFT) -> np.ndarray:
    """faster-whisper FeatureExtractor.get_mel_filters: slaney-scale triangles, slaney norm."""
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mels = np.linspace(0.0, 45.245640471924965, n_mels + 2)
    f_sp = 200.0 / 3
    freqs = f_sp * mels
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    log_t = mels >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (mels[log_t] - min_log_mel))
    fdiff = np.diff(freqs)
    ramps = freqs.reshape(-1, 1) - fftfreqs.reshape(1, -1)
    lower = -ramps[:-2] / fdiff[:-1].reshape(-1, 1)
    upper = ramps[2:] / fdiff[1:].reshape(-1, 1)
    weights = np.maximum(0.0, np.minimum(lower, upper))
    enorm = 2.0 / (freqs[2: n_mels + 2] - freqs[:n_mels])
    return weights * enorm[:, None]


def reflect_index(idx: np.ndarray, n: int) -> np.ndarray:
    """numpy 'reflect' padding index map (iterated reflection = periodic mirror, period 2(n-1))."""
    if n == 1:
        return np.zeros_like(idx)
    p = 2 * (n - 1)
    m = np.mod(idx, p)
    return np.where(m < n, m, p - m)


def logmel_frames(audio: np.ndarray, n_mels: int) -> np.ndarray:
    """Un-normalised log10 mel for faster-whisper's framing: audio + 160 zeros, centre reflect pad,
    periodic Hann 400, hop 160, |rfft|^2, drop last frame.  Returns [n_mels, F], F = N//160 + 1."""
    x = np.concatenate([np.asarray(audio, dtype=np.float64), np.zeros(HOP)])
    L = x.shape[0]
    n_frames = 1 + L // HOP
    idx = np.arange(n_frames)[:, None] * HOP + np.arange(N_FFT)[None, :] - N_FFT // 2
    frames = x[reflect_index(idx, L)]
    window = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(N_FFT) / N_FFT)
    spec = np.fft.rfft(frames * window[None, :], axis=-1)
    power = (spec.real ** 2 + spec.imag ** 2)[:-1]  # drop last frame -> [F, 201]
    mel = power @ mel_filters(n_mels).T
    return np.log10(np.maximum(mel, 1e-10)).T  # [M, F]


def logmel(audio: np.ndarray, n_mels: int) -> np.ndarray:
    """faster-whisper FeatureExtractor(...)(audio): normalised features [n_mels, N//160 + 1]."""
    lm = logmel_frames(audio, n_mels)
    lm = np.maximum(lm, lm.max() - 8.0)
    return ((lm + 4.0) / 4.0).astype(np.float32)


def logmel_segment(audio: np.ndarray, n_mels: int, seek: int = 0) -> np.ndarray:
    """The encoder input of one window, faster-whisper generate_segments: content_frames = F - 1,
    segment = features[:, seek : seek + min(3000, content_frames - seek)], pad_or_trim to 3000."""
    feats = logmel(audio, n_mels)
    content = feats.shape[1] - 1
    size = max(0, min(N_FRAMES, content - seek))
    seg = np.zeros((n_mels, N_FRAMES), dtype=np.float32)
    seg[:, :size] = feats[:, seek: seek + size]
    return seg


# ----------------------------------------------------------------------------------------------
# transformer blocks
# ----------------------------------------------------------------------------------------------
def gelu(x):
    return (0.5 * x * (1.0 + erf(x / np.float32(math.sqrt(2.0))))).astype(np.float32)


def layer_norm(x, g, b, eps=1e-5):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return ((x - mu) / np.sqrt(var + eps) * g + b).astype(np.float32)


def linear(x, W, p, bias=True):
    y = x @ W[p + ".weight"].T
    if bias:
        y = y + W[p + ".bias"]
    return y.astype(np.float32)


def softmax(x, axis=-1):
    m = np.max(x, axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def mha(q, k, v, n_head, mask=None, return_probs=False):
    """q [Tq,d], k/v [Tk,d]; softmax(q k^T / sqrt(dh)) v per head."""
    Tq, dm = q.shape
    dh = dm // n_head
    qh = q.reshape(Tq, n_head, dh).transpose(1, 0, 2)
    kh = k.reshape(-1, n_head, dh).transpose(1, 0, 2)
    vh = v.reshape(-1, n_head, dh).transpose(1, 0, 2)
    s = (qh @ kh.transpose(0, 2, 1)) * np.float32(dh ** -0.5)
    if mask is not None:
        s = s + mask
    p = softmax(s, -1).astype(np.float32)
    o = (p @ vh).transpose(1, 0, 2).reshape(Tq, dm).astype(np.float32)
    return (o, s) if return_probs else o


def conv1d_k3(x, w, b, stride):
    """x [C,T], w [O,C,3], padding 1."""
    C, T = x.shape
    xp = np.pad(x, ((0, 0), (1, 1)))
    Tout = (T + 2 - 3) // stride + 1
    cols = np.stack([xp[:, k: k + stride * (Tout - 1) + 1: stride] for k in range(3)], axis=0)  # [3,C,Tout]
    y = np.einsum("ock,kct->ot", w, cols, optimize=True) + b[:, None]
    return y.astype(np.float32)


def encoder(W, d: Dims, mel: np.ndarray, mx8: bool = False) -> np.ndarray:
    """WhisperEncoder.forward (modeling_whisper.py:592): conv-GELU x2, + sinusoid, L pre-LN blocks, LN.
    mx8: the four projections of every layer take MX-fp8-quantized operands (model dtype float8 / config 5)."""
    lin = linear_mx8 if mx8 else linear
    x = gelu(conv1d_k3(mel.astype(np.float32), W["encoder.conv1.weight"], W["encoder.conv1.bias"], 1))
    x = gelu(conv1d_k3(x, W["encoder.conv2.weight"], W["encoder.conv2.bias"], 2))
    x = (x.T + W["encoder.embed_positions.weight"][: x.shape[1]]).astype(np.float32)
    for i in range(d.n_audio_layer):
        p = f"encoder.layers.{i}"
        h = layer_norm(x, W[p + ".self_attn_layer_norm.weight"], W[p + ".self_attn_layer_norm.bias"])
        q = lin(h, W, p + ".self_attn.q_proj")
        k = lin(h, W, p + ".self_attn.k_proj", bias=False)
        v = lin(h, W, p + ".self_attn.v_proj")
        x = x + lin(mha(q, k, v, d.n_audio_head), W, p + ".self_attn.out_proj")
        h = layer_norm(x, W[p + ".final_layer_norm.weight"], W[p + ".final_layer_norm.bias"])
        x = x + lin(gelu(lin(h, W, p + ".fc1")), W, p + ".fc2")
    return layer_norm(x, W["encoder.layer_norm.weight"], W["encoder.layer_norm.bias"])


class DecoderCache:
    """Per-sequence self-attention KV cache + the window's cross K/V (openai-whisper kv_cache)."""

    def __init__(self, W, d: Dims, enc: np.ndarray):
        self.d = d
        self.k = [np.zeros((0, d.n_text_state), np.float32) for _ in range(d.n_text_layer)]
        self.v = [np.zeros((0, d.n_text_state), np.float32) for _ in range(d.n_text_layer)]
        self.ck, self.cv = [], []
        kv8 = bool(W.get("decoder.kv8", False))  # the fp8 decode's image rule (fp8_decoder_weights)
        for i in range(d.n_text_layer):
            p = f"decoder.layers.{i}.encoder_attn"
            k, v = linear(enc, W, p + ".k_proj", bias=False), linear(enc, W, p + ".v_proj")
            if kv8:
                k, v = kv8_images(k, d.n_text_head), kv8_images(v, d.n_text_head)
            self.ck.append(k)
            self.cv.append(v)

    @property
    def length(self):
        return self.k[0].shape[0]

    def copy(self):
        c = DecoderCache.__new__(DecoderCache)
        c.d, c.ck, c.cv = self.d, self.ck, self.cv
        c.k = [a.copy() for a in self.k]
        c.v = [a.copy() for a in self.v]
        return c


def decoder_forward(W, d: Dims, tokens, cache: DecoderCache, align_heads=None):
    """WhisperDecoder.forward (modeling_whisper.py:690) for new `tokens` appended after the cache.
    Returns logits [T, V] (and cross-attention pre-softmax scores of `align_heads` as [n, T, 1500])."""
    tokens = np.asarray(tokens, dtype=np.int64)
    T = tokens.shape[0]
    off = cache.length
    x = (W["decoder.embed_tokens.weight"][tokens] + W["decoder.embed_positions.weight"][off: off + T]).astype(np.float32)
    causal = np.triu(np.full((T, off + T), -np.inf, np.float32), k=off + 1)
    qk_store = []
    for i in range(d.n_text_layer):
        p = f"decoder.layers.{i}"
        h = layer_norm(x, W[p + ".self_attn_layer_norm.weight"], W[p + ".self_attn_layer_norm.bias"])
        q = linear(h, W, p + ".self_attn.q_proj")
        cache.k[i] = np.concatenate([cache.k[i], linear(h, W, p + ".self_attn.k_proj", bias=False)])
        cache.v[i] = np.concatenate([cache.v[i], linear(h, W, p + ".self_attn.v_proj")])
        x = x + linear(mha(q, cache.k[i], cache.v[i], d.n_text_head, causal), W, p + ".self_attn.out_proj")
        h = layer_norm(x, W[p + ".encoder_attn_layer_norm.weight"], W[p + ".encoder_attn_layer_norm.bias"])
        q = linear(h, W, p + ".encoder_attn.q_proj")
        o, s = mha(q, cache.ck[i], cache.cv[i], d.n_text_head, return_probs=True)
        if align_heads is not None:
            for (l, hh) in align_heads:
                if l == i:
                    qk_store.append(s[hh])
        x = x + linear(o, W, p + ".encoder_attn.out_proj")
        h = layer_norm(x, W[p + ".final_layer_norm.weight"], W[p + ".final_layer_norm.bias"])
        x = x + linear(gelu(linear(h, W, p + ".fc1")), W, p + ".fc2")
    x = layer_norm(x, W["decoder.layer_norm.weight"], W["decoder.layer_norm.bias"])
    # (the fp8 decode's logits projection is the quantized embedding, fp8_decoder_weights)
    logits = (x @ W.get("decoder.proj_out.weight", W["decoder.embed_tokens.weight"]).T).astype(np.float32)
    if align_heads is not None:
        return logits, np.stack(qk_store) if qk_store else np.zeros((0, T, cache.ck[0].shape[0]), np.float32)
    return logits


# ----------------------------------------------------------------------------------------------
# decoding rules (openai-whisper decoding.py LogitFilters; CT2 re-implements the same rules)
# ----------------------------------------------------------------------------------------------
@dataclass
class DecodeOptions:
    task: str = "transcribe"
    language: int | None = None          # language token id, None = detect
    beam_size: int = 1                    # 1 = greedy (temperature 0)
    patience: float = 1.0
    length_penalty: float | None = None   # None/1.0 -> logprob / len (CT2 length_penalty=1)
    max_new_tokens: int = 224
    suppress_blank: bool = True
    suppress_tokens: tuple = ()
    without_timestamps: bool = False
    max_initial_timestamp_index: int | None = 50


def apply_rules(logits: np.ndarray, sampled: list, sp: Special, opt: DecodeOptions) -> np.ndarray:
    """SuppressBlank -> SuppressTokens -> ApplyTimestampRules for ONE row; `sampled` = tokens generated
    after the SOT sequence.  Returns filtered float32 logits (-inf masked)."""
    x = logits.astype(np.float32).copy()
    V = x.shape[0]
    if opt.suppress_blank and len(sampled) == 0:
        x[[sp.blank, sp.eot]] = -np.inf
    if opt.suppress_tokens:
        x[list(opt.suppress_tokens)] = -np.inf
    if opt.without_timestamps:
        x[sp.no_timestamps] = -np.inf  # the SOT sequence carries <|notimestamps|>; rules below skipped
        return x
    tb = sp.timestamp_begin
    x[sp.no_timestamps] = -np.inf
    last_ts = len(sampled) >= 1 and sampled[-1] >= tb
    pen_ts = len(sampled) < 2 or sampled[-2] >= tb
    if last_ts:
        if pen_ts:
            x[tb:] = -np.inf
        else:
            x[: sp.eot] = -np.inf
    ts = [t for t in sampled if t >= tb]
    if ts:
        ts_last = ts[-1] if (last_ts and not pen_ts) else ts[-1] + 1
        x[tb: ts_last] = -np.inf
    if len(sampled) == 0:
        x[:tb] = -np.inf
        if opt.max_initial_timestamp_index is not None:
            x[tb + opt.max_initial_timestamp_index + 1:] = -np.inf
    lp = log_softmax(x)
    ts_lp = logsumexp(lp[tb:])
    if ts_lp > np.max(lp[:tb]):
        x[:tb] = -np.inf
    return x


def log_softmax(x):
    x = x.astype(np.float64)
    m = np.max(x)
    if not np.isfinite(m):
        return np.full_like(x, -np.inf)
    return (x - m - np.log(np.sum(np.exp(x - m)))).astype(np.float64)


def logsumexp(x):
    x = np.asarray(x, np.float64)
    m = np.max(x)
    if not np.isfinite(m):
        return -np.inf
    return float(m + np.log(np.sum(np.exp(x - m))))


def sot_sequence(sp: Special, language: int, task: str, without_timestamps=False):
    seq = [sp.sot, language, sp.translate if task == "translate" else sp.transcribe]
    if without_timestamps:
        seq.append(sp.no_timestamps)
    return seq


def build_prompt(sp: Special, prompt_ids, language, task, without_timestamps=False, max_prompt=223):
    """faster-whisper get_prompt: [<|startofprev|>] + last (448//2 - 1) prompt ids + SOT sequence."""
    pre = []
    if prompt_ids:
        pre = [sp.sot_prev] + list(prompt_ids)[-max_prompt:]
    return pre + sot_sequence(sp, language, task, without_timestamps)


def detect_language(W, d: Dims, enc: np.ndarray):
    """openai-whisper detect_language / CT2 Whisper.detect_language: logits at <|startoftranscript|>,
    restricted to language tokens.  Returns (lang_token, prob)."""
    sp = special_tokens(d.n_vocab)
    cache = DecoderCache(W, d, enc)
    logits = decoder_forward(W, d, [sp.sot], cache)[0]
    lang = logits[sp.lang0: sp.lang0 + sp.n_langs].astype(np.float64)
    p = np.exp(lang - lang.max())
    p /= p.sum()
    i = int(np.argmax(lang))
    return sp.lang0 + i, float(p[i])


@dataclass
class DecodeResult:
    tokens: list          # sampled tokens (without the trailing EOT)
    sum_logprob: float
    avg_logprob: float    # sum_logprob / (len(tokens) + 1)  (faster-whisper generate_with_fallback)
    no_speech_prob: float
    language: int


def decode(W, d: Dims, enc: np.ndarray, opt: DecodeOptions, prompt_ids=(), forced=None):
    """Greedy (beam_size == 1) or beam search over one window.  `forced` = teacher-forced token list
    (greedy only): the argmax/margin per step is recorded instead of being fed back."""
    sp = special_tokens(d.n_vocab)
    lang = opt.language
    if lang is None:
        lang, _ = detect_language(W, d, enc)
    prefix = build_prompt(sp, list(prompt_ids), lang, opt.task, opt.without_timestamps)
    sot_index = prefix.index(sp.sot)
    base = DecoderCache(W, d, enc)
    logits = decoder_forward(W, d, prefix, base)
    no_speech = float(softmax(logits[sot_index].astype(np.float64))[sp.no_speech])
    max_new = min(opt.max_new_tokens, d.n_text_ctx - len(prefix))
    if opt.beam_size <= 1:
        return _greedy(W, d, sp, opt, base, logits[-1], no_speech, lang, max_new, forced)
    return _beam(W, d, sp, opt, base, logits[-1], no_speech, lang, max_new)


def forced_rows(W, d: Dims, encs, prefix, tokens, parents, K: int, keep=None):
    """Teacher-forced decoding of R = len(encs) x K rows (row r belongs to window r // K), the beam bookkeeping of
    openai BeamSearchDecoder.update (decoding.py: each new row continues the KV cache of its source row):
    every row starts from prefix[b]; step i appends tokens[i][r] to the sequence of row parents[i][r].
    Returns (top1 [n+1][R], top-2 margin [n+1][R], {step: logits [R][V]} for the steps in `keep`), step 0 = the
    prefix's last position."""
    R = len(encs) * K
    n = len(tokens)
    keep = set(range(n + 1)) if keep is None else set(keep)
    caches, last = [], []
    for b, enc in enumerate(encs):
        c = DecoderCache(W, d, enc)
        lg = decoder_forward(W, d, list(prefix[b]), c)[-1]
        for _ in range(K):
            caches.append(c.copy())
            last.append(lg)
    top1 = np.zeros((n + 1, R), np.int64)
    margin = np.zeros((n + 1, R), np.float32)
    out = {}
    for i in range(n + 1):
        L = np.stack(last)
        top1[i] = np.argmax(L, axis=-1)
        t2 = np.partition(L, -2, axis=-1)[:, -2:]
        margin[i] = t2[:, 1] - t2[:, 0]
        if i in keep:
            out[i] = L
        if i == n:
            break
        new_c = [caches[int(parents[i][r])].copy() for r in range(R)]
        last = [decoder_forward(W, d, [int(tokens[i][r])], new_c[r])[0] for r in range(R)]
        caches = new_c
    return top1, margin, out


def _greedy(W, d, sp, opt, cache, last_logits, no_speech, lang, max_new, forced):
    sampled, total, trace = [], 0.0, []
    cur = last_logits
    for step in range(max_new):
        x = apply_rules(cur, sampled, sp, opt)
        lp = log_softmax(x)
        order = np.argsort(-x, kind="stable")
        tok = int(order[0])
        margin = float(x[order[0]] - x[order[1]]) if np.isfinite(x[order[1]]) else np.inf
        trace.append((tok, margin))
        if forced is not None:
            if step >= len(forced):
                break
            tok = int(forced[step])
        total += float(lp[tok])
        if tok == sp.eot:
            break
        sampled.append(tok)
        cur = decoder_forward(W, d, [tok], cache)[0]
    res = DecodeResult(sampled, total, total / (len(sampled) + 1), no_speech, lang)
    res.trace = trace
    return res


def _beam(W, d, sp, opt, cache0, last_logits, no_speech, lang, max_new):
    """openai-whisper BeamSearchDecoder (patience) + MaximumLikelihoodRanker; ties broken by
    (score desc, source beam asc, token asc) — deterministic, mirrored by the HIP kernel."""
    K = opt.beam_size
    max_cand = int(round(K * opt.patience))
    beams = [([], 0.0, cache0.copy(), last_logits) for _ in range(K)]
    finished = {}
    trace = []
    for step in range(max_new):
        cands = []
        seen = set()
        for j, (seq, score, cache, lg) in enumerate(beams):
            x = apply_rules(lg, seq, sp, opt)
            lp = log_softmax(x)
            top = np.lexsort((np.arange(lp.shape[0]), -lp))[: K + 1]
            for t in top:
                s = tuple(seq + [int(t)])
                if s in seen:
                    continue
                seen.add(s)
                cands.append((score + float(lp[t]), j, int(t), s))
        cands.sort(key=lambda c: (-c[0], c[1], c[2]))
        new_beams, new_fin = [], []
        used = 0
        for sc, j, t, s in cands:
            used += 1
            if t == sp.eot:
                new_fin.append((s, sc))
            else:
                new_beams.append((list(s), sc, j))
                if len(new_beams) == K:
                    break
        # selection margin of this step: the smallest score gap among the candidates that decided it and the first
        # one left out (a perturbation below it cannot change which hypotheses survive, nor their order)
        sc_used = [c[0] for c in cands[: used + 1]]
        trace.append(min([a - b for a, b in zip(sc_used, sc_used[1:])], default=np.inf))
        for s, sc in new_fin:
            if len(finished) >= max_cand:
                break
            if s not in finished:
                finished[s] = sc
        if len(finished) >= max_cand or step == max_new - 1:
            beams = [(s, sc, beams[j][2], None) for (s, sc, j) in new_beams]
            break
        nb = []
        for s, sc, j in new_beams:
            c = beams[j][2].copy()
            lg = decoder_forward(W, d, [s[-1]], c)[0]
            nb.append((s, sc, c, lg))
        beams = nb
    if len(finished) < K:
        for s, sc, _, _ in sorted(beams, key=lambda b: -b[1]):
            key = tuple(s) + (sp.eot,)
            if key not in finished:
                finished[key] = sc
            if len(finished) >= K:
                break
    best, best_score, best_sum = None, -np.inf, 0.0
    norms = []
    for s, sc in finished.items():
        toks = [t for t in s if t != sp.eot]
        L = max(len(toks), 1)  # openai ranks the sequence trimmed at EOT (decoding.py DecodingTask.run)
        pen = L if opt.length_penalty is None else ((5 + L) / 6) ** opt.length_penalty
        norm = sc / pen
        norms.append(norm)
        if norm > best_score:
            best, best_score, best_sum = toks, norm, sc
    res = DecodeResult(best, best_sum, best_sum / (len(best) + 1), no_speech, lang)
    res.trace = trace  # per step: selection margin (see above)
    norms.sort(reverse=True)
    res.final_margin = norms[0] - norms[1] if len(norms) > 1 else np.inf  # ranking margin of the chosen sequence
    return res


def topk_stable(lp, k: int):
    """The k best ids by (value desc, id asc) -- np.lexsort((ids, -lp))[:k] -- via a partition (same result)."""
    thr = np.partition(lp, -k)[-k]
    c = np.nonzero(lp >= thr)[0]
    return c[np.lexsort((c, -lp[c]))][:k]


def _ts_rule_gap(x, sp: Special, opt: DecodeOptions) -> float:
    """|logsumexp(timestamp log-probs) - max(text log-prob)| of apply_rules' last rule, on the logits it sees."""
    if opt.without_timestamps:
        return np.inf
    lp = log_softmax(x)
    tb = sp.timestamp_begin
    a, b = logsumexp(lp[tb:]), np.max(lp[:tb])
    if not (np.isfinite(a) and np.isfinite(b)):
        return np.inf
    return abs(a - b)


def search_replay(logits, sel, K: int, sp: Special, opt: DecodeOptions, eps: float = 1e-3):
    """The decode SEARCH of _greedy / _beam, replayed on recorded per-step logits (wmx_ctx_record: logits [n][R][V]
    of the R = windows x K rows, the device's selection sel [n][R][2]) so the rules, top-k, beam bookkeeping and
    finished-hypothesis handling are checked token-exactly over every recorded step, independent of the 16-bit
    noise in the logits.  Per window the replay compares its own selection with the device's at every step; a
    disagreement at a step whose deciding score gap (or timestamp-rule gap) is below `eps` is a legitimate
    float tie (f32 device log-softmax vs f64 here) and ends that window's comparison.
    Returns per window dict(steps=compared steps, ties=bool, mismatch=None or (step, ours, device),
    finished=[(tokens, score)], alive=[(tokens, score)])."""
    n, R, _ = logits.shape
    B = R // K
    out = []
    for b in range(B):
        rows = range(b * K, (b + 1) * K)
        info = dict(steps=0, ties=False, mismatch=None, finished=[], alive=[])
        if K == 1:
            r, seq, total = b, [], 0.0
            for i in range(n):
                dev = tuple(sel[i][r])
                if dev[0] < 0:
                    break
                x = apply_rules(logits[i][r], seq, sp, opt)
                order = np.argsort(-x, kind="stable")
                tok = int(order[0])
                gap = min(float(x[order[0]] - x[order[1]]), _ts_rule_gap(logits[i][r], sp, opt))
                if tok != dev[1]:
                    if gap <= eps:
                        info["ties"] = True
                    else:
                        info["mismatch"] = (i, tok, dev[1])
                    break
                info["steps"] += 1
                total += float(log_softmax(x)[tok])
                if tok == sp.eot:
                    info["finished"].append((list(seq), total))
                    break
                seq.append(tok)
            if not info["finished"]:
                info["alive"].append((list(seq), total))
            out.append(info)
            continue
        max_cand = int(round(K * opt.patience))
        beams = [([], 0.0) for _ in range(K)]
        finished = {}
        for i in range(n):
            dev = [tuple(sel[i][r]) for r in rows]
            if dev[0][0] < 0:
                break
            cands = []
            gap_rule = np.inf
            for j, (seq, score) in enumerate(beams if i > 0 else beams[:1]):
                lg = logits[i][b * K + j]
                x = apply_rules(lg, seq, sp, opt)
                gap_rule = min(gap_rule, _ts_rule_gap(lg, sp, opt))
                lp = log_softmax(x)
                cands += [(score + float(lp[t]), j, int(t)) for t in topk_stable(lp, K + 1)]
            cands.sort(key=lambda c: (-c[0], c[1], c[2]))
            new_beams, new_fin, used = [], [], 0
            for sc, j, t in cands:
                used += 1
                if t == sp.eot:
                    new_fin.append((beams[j][0], sc))
                else:
                    new_beams.append((beams[j][0] + [t], sc, j))
                    if len(new_beams) == K:
                        break
            scs = [c[0] for c in cands[: used + 1]]
            gap = min([gap_rule] + [a - c for a, c in zip(scs, scs[1:])])
            ours = [(b * K + j, s[-1]) for s, _, j in new_beams]
            if ours != dev[: len(ours)]:
                if gap <= eps:
                    info["ties"] = True
                else:
                    info["mismatch"] = (i, ours, dev)
                break
            info["steps"] += 1
            for s, sc in new_fin:
                if len(finished) >= max_cand:
                    break
                finished.setdefault(tuple(s), sc)
            beams = [(s, sc) for s, sc, _ in new_beams]
            if len(finished) >= max_cand:
                break
        info["finished"] = [(list(s), sc) for s, sc in finished.items()]
        info["alive"] = [(list(s), sc) for s, sc in beams]
        out.append(info)
    return out


def sample_gumbel(seed: int, row: int, slot: int, toks) -> np.ndarray:
    """The device's sampling noise (csrc/wmx_decode.hip sample_gumbel), bit for bit up to the two f32 logs:
    splitmix64 of ((row * 1024 + slot) * 65536 + token) + seed * 0x9E3779B97F4A7C15, u = (top 23 bits * 2 + 1) / 2^25,
    Gumbel = -log(-log(u)) in float32."""
    g = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        t = np.asarray(toks, np.uint64)
        base = (np.uint64(row) * np.uint64(1024) + np.uint64(slot)) * np.uint64(65536)
        z = t + base + np.array([seed], np.uint64) * g
        z = z + g
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = ((z >> np.uint64(41)).astype(np.uint32) * np.uint32(2) + np.uint32(1)).astype(np.float32) * np.float32(2.0 ** -25)
    return -np.log(-np.log(u))


def sampling_replay(logits, sel, K: int, sp: Special, opt: DecodeOptions, temperature: float, seed: int, slot0: int,
                    eps: float = 1e-3):
    """faster-whisper's T > 0 branch (CT2 generate with beam_size 1, num_hypotheses = best_of = K, sampling_topk 0,
    sampling_temperature = T), replayed on the recorded logits of wmx_ctx_record: every row independently draws
    argmax(rule-masked logits / T + Gumbel) with the device's noise (sample_gumbel, slot = slot0 + step), accumulates
    the rule-masked log-softmax of the UNSCALED logits (openai DecodingTask: logprobs before the temperature), and
    each window keeps the row with the best sum_logprob / length.  A draw that differs from the device's at a step
    whose top-2 key gap is <= eps is an f32 tie and ends that row's comparison.  Returns per window
    dict(rows=[dict(steps, ties, mismatch, tokens, total, finished)], best=(row, tokens, total) or None)."""
    n, R, V = logits.shape
    inv_t = np.float32(1.0 / temperature)
    out = []
    for b in range(R // K):
        rows = []
        for j in range(K):
            r = b * K + j
            info = dict(steps=0, ties=False, mismatch=None, tokens=[], total=0.0, finished=False)
            for i in range(n):
                dev = tuple(sel[i][r])
                if dev[0] < 0:
                    break
                x = apply_rules(logits[i][r], info["tokens"], sp, opt)
                ok = np.isfinite(x)
                key = np.full(V, -np.inf, np.float32)
                key[ok] = x[ok].astype(np.float32) * inv_t + sample_gumbel(seed, r, slot0 + i, np.nonzero(ok)[0])
                order = np.argsort(-key, kind="stable")
                tok = int(order[0])
                gap = min(float(key[order[0]] - key[order[1]]), _ts_rule_gap(logits[i][r], sp, opt))
                if tok != dev[1]:
                    if gap <= eps:
                        info["ties"] = True
                    else:
                        info["mismatch"] = (i, tok, dev[1])
                    break
                info["steps"] += 1
                info["total"] += float(log_softmax(x)[tok])
                if tok == sp.eot:
                    info["finished"] = True
                    break
                info["tokens"].append(tok)
            rows.append(info)
        best = None
        if not any(rw["ties"] or rw["mismatch"] for rw in rows):
            sc = [rw["total"] / max(len(rw["tokens"]), 1) for rw in rows]
            jb = int(np.argmax(sc))
            best = (jb, rows[jb]["tokens"], rows[jb]["total"])
        out.append(dict(rows=rows, best=best))
    return out


def rank_final(finished, alive, K: int, length_penalty=None):
    """openai BeamSearchDecoder.finalize (fill the finished list from the best alive beams) +
    MaximumLikelihoodRanker; returns (tokens, sum_logprob, ranking margin to the runner-up)."""
    fin = dict((tuple(s), sc) for s, sc in finished)
    for s, sc in sorted(alive, key=lambda a: -a[1]):
        if len(fin) >= K:
            break
        fin.setdefault(tuple(s), sc)
    scored = []
    for s, sc in fin.items():
        L = max(len(s), 1)
        pen = L if length_penalty is None else ((5 + L) / 6) ** length_penalty
        scored.append((sc / pen, list(s), sc))
    scored.sort(key=lambda a: -a[0])
    margin = scored[0][0] - scored[1][0] if len(scored) > 1 else np.inf
    return scored[0][1], scored[0][2], margin


# ----------------------------------------------------------------------------------------------
# word-level alignment (openai-whisper timing.py find_alignment / faster-whisper find_alignment)
# ----------------------------------------------------------------------------------------------
def median_filter(x: np.ndarray, width: int) -> np.ndarray:
    """openai timing.median_filter: reflect-pad the last axis by width//2, sliding median."""
    pad = width // 2
    if x.shape[-1] <= pad:
        return x
    xp = np.pad(x, [(0, 0)] * (x.ndim - 1) + [(pad, pad)], mode="reflect")
    win = np.lib.stride_tricks.sliding_window_view(xp, width, axis=-1)
    return np.sort(win, axis=-1)[..., pad]


def dtw(cost: np.ndarray):
    """openai timing.dtw_cpu + backtrace: returns (text_indices, time_indices)."""
    N, M = cost.shape
    c = np.full((N + 1, M + 1), np.inf, np.float32)
    tr = -np.ones((N + 1, M + 1), np.float32)
    c[0, 0] = 0
    for j in range(1, M + 1):
        for i in range(1, N + 1):
            c0, c1, c2 = c[i - 1, j - 1], c[i - 1, j], c[i, j - 1]
            if c0 < c1 and c0 < c2:
                v, t = c0, 0
            elif c1 < c0 and c1 < c2:
                v, t = c1, 1
            else:
                v, t = c2, 2
            c[i, j] = cost[i - 1, j - 1] + v
            tr[i, j] = t
    i, j = N, M
    tr[0, :] = 2
    tr[:, 0] = 1
    ti, tj = [], []
    while i > 0 or j > 0:
        ti.append(i - 1)
        tj.append(j - 1)
        t = tr[i, j]
        if t == 0:
            i -= 1
            j -= 1
        elif t == 1:
            i -= 1
        else:
            j -= 1
    return np.array(ti[::-1]), np.array(tj[::-1])


def alignment_heads_default(d: Dims):
    """openai Whisper.alignment_heads default: every head of the second half of the decoder."""
    return [(l, h) for l in range(d.n_text_layer // 2, d.n_text_layer) for h in range(d.n_text_head)]


def find_alignment(W, d: Dims, enc: np.ndarray, language: int, task: str, text_tokens, num_frames: int,
                   align_heads=None, medfilt_width: int = 7, return_matrix: bool = False):
    """Returns (text_indices, time_indices, text_token_probs, jump_times) for the token sequence
    sot_sequence + [<|notimestamps|>] + text + [eot] (openai timing.find_alignment); with return_matrix, also the
    matrix the DTW runs on ([len(text) + 1][num_frames // 2], before the sign flip)."""
    sp = special_tokens(d.n_vocab)
    heads = align_heads if align_heads is not None else alignment_heads_default(d)
    sot = sot_sequence(sp, language, task)
    tokens = sot + [sp.no_timestamps] + list(text_tokens) + [sp.eot]
    cache = DecoderCache(W, d, enc)
    logits, qk = decoder_forward(W, d, tokens, cache, align_heads=heads)
    sampled = logits[len(sot):, : sp.eot].astype(np.float64)
    probs = softmax(sampled, -1)
    text_token_probs = probs[np.arange(len(text_tokens)), list(text_tokens)] if text_tokens else np.zeros(0)
    w = qk[:, :, : num_frames // 2].astype(np.float64)
    w = softmax(w, -1)
    std = w.std(axis=-2, keepdims=True)
    mean = w.mean(axis=-2, keepdims=True)
    w = (w - mean) / std
    w = median_filter(w, medfilt_width)
    matrix = w.mean(axis=0)[len(sot): -1]
    ti, tj = dtw(-matrix.astype(np.float32))
    jumps = np.pad(np.diff(ti), (1, 0), constant_values=1).astype(bool)
    jump_times = tj[jumps] / 50.0
    if return_matrix:
        return ti, tj, text_token_probs, jump_times, matrix
    return ti, tj, text_token_probs, jump_times
