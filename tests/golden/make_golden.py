"""Generate the golden fixtures that pin the CPU oracle (run in the build container only).

The reference repo ships no tests or fixtures and its arithmetic lives in un-vendored packages
(faster-whisper 1.2.1 / CTranslate2 4.6.1).  The only independent Whisper
implementation available offline is transformers 5.15.0, so the oracle is pinned against it:

* log-mel: ``WhisperFeatureExtractor._np_extract_fbank_features`` applied to ``audio + 160 zeros``
  (= faster-whisper's ``padding=160`` framing; HF's STFT/filterbank/log10/max-8/(x+4)/4 are the same
  published algorithm).
* encoder output, decoder logits (teacher forced) and cross-attention scores: ``WhisperForConditionalGeneration``
  loaded with the build-owned synthetic weights (oracle.whisper_np.make_weights).
* decode rules: ``SuppressTokensAtBeginLogitsProcessor``, ``SuppressTokensLogitsProcessor``,
  ``WhisperTimeStampLogitsProcessor``.
* DTW / median filter: ``generation_whisper._dynamic_time_warping`` / ``_median_filter``.

Only data (inputs and expected outputs) is written; audio is regenerated from its seed and checked by
sha256.  Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "realtime-whisper-asr_amd"))

from oracle import whisper_np as O  # noqa: E402
from wmx import synth  # noqa: E402

AUDIO_CASES = [  # (name, kind, seed, seconds)
    ("sp_0p5", "speech", 11, 0.5),
    ("sp_1", "speech", 12, 1.0),
    ("sp_7p3", "speech", 13, 7.3),
    ("noise_4", "noise", 14, 4.0),
    ("zeros_2", "zeros", 0, 2.0),
    ("sp_30", "speech", 15, 30.0),
    ("sp_31", "speech", 16, 31.0),
]


def make_audio(kind, seed, seconds):
    n = int(round(seconds * 16000))
    if kind == "speech":
        return synth.speech_like(seed, n)
    if kind == "noise":
        return synth.white_noise(seed, n)
    return np.zeros(n, np.float32)


def hf_logmel(audio, n_mels):
    from transformers import WhisperFeatureExtractor
    fe = WhisperFeatureExtractor(feature_size=n_mels)
    return fe._np_extract_fbank_features(np.pad(audio, (0, 160))[None], "cpu")[0]


def gen_logmel(out):
    for name, kind, seed, sec in AUDIO_CASES:
        a = make_audio(kind, seed, sec)
        out[f"logmel/{name}/sha"] = np.frombuffer(synth.digest(a).encode(), dtype=np.uint8)
        for m in (80, 128):
            ref = hf_logmel(a, m).astype(np.float32)
            if ref.shape[1] > 800:  # keep the fixture small: every 7th frame + the last 3
                idx = np.unique(np.concatenate([np.arange(0, ref.shape[1], 7), np.arange(ref.shape[1] - 3, ref.shape[1])]))
            else:
                idx = np.arange(ref.shape[1])
            out[f"logmel/{name}/{m}/frames"] = idx.astype(np.int32)
            out[f"logmel/{name}/{m}/value"] = ref[:, idx]
            out[f"logmel/{name}/{m}/nframes"] = np.int32(ref.shape[1])


def hf_model(d: O.Dims, W):
    from transformers import WhisperConfig, WhisperForConditionalGeneration
    cfg = WhisperConfig(vocab_size=d.n_vocab, num_mel_bins=d.n_mels, encoder_layers=d.n_audio_layer,
                        encoder_attention_heads=d.n_audio_head, decoder_layers=d.n_text_layer,
                        decoder_attention_heads=d.n_text_head, d_model=d.n_audio_state,
                        encoder_ffn_dim=4 * d.n_audio_state, decoder_ffn_dim=4 * d.n_text_state,
                        max_source_positions=d.n_audio_ctx, max_target_positions=d.n_text_ctx,
                        activation_function="gelu", scale_embedding=False, dropout=0.0,
                        attention_dropout=0.0, activation_dropout=0.0)
    cfg._attn_implementation = "eager"
    m = WhisperForConditionalGeneration(cfg).eval()
    sd = {("model." + k): torch.from_numpy(np.ascontiguousarray(v)) for k, v in W.items()}
    sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k == "proj_out.weight" for k in missing), missing
    return m


def gen_model(out, name, seed, dtype):
    d = O.DIMS[name]
    W = O.make_weights(d, seed, dtype)
    m = hf_model(d, W)
    sp = O.special_tokens(d.n_vocab)
    a = make_audio("speech", 21, 7.3)
    mel = O.logmel_segment(a, d.n_mels)
    key = f"model/{name}/{dtype}/{seed}"
    with torch.no_grad():
        enc = m.model.encoder(torch.from_numpy(mel)[None]).last_hidden_state[0].numpy()
    rows = np.arange(0, d.n_audio_ctx, 5)
    out[key + "/enc_rows"] = rows.astype(np.int32)
    out[key + "/enc"] = enc[rows]
    # teacher-forced decoder: prompt + SOT + a few text/timestamp tokens
    toks = [sp.sot_prev, 440, 1000, sp.sot, sp.lang0, sp.transcribe, sp.timestamp_begin, 2425, 11, 50, 3000,
            sp.timestamp_begin + 12, sp.timestamp_begin + 12, 777]
    out[key + "/dec_tokens"] = np.array(toks, np.int32)
    with torch.no_grad():
        r = m.model.decoder(input_ids=torch.tensor([toks]), encoder_hidden_states=torch.from_numpy(enc)[None],
                            output_attentions=True)
        logits = (r.last_hidden_state[0] @ m.model.decoder.embed_tokens.weight.T).numpy()
    probe = np.unique(np.concatenate([np.random.default_rng(5).integers(0, d.n_vocab, 512),
                                      np.arange(sp.eot, d.n_vocab, 37)])).astype(np.int32)
    out[key + "/dec_probe"] = probe
    out[key + "/dec_logits_probe"] = logits[:, probe]
    out[key + "/dec_argmax"] = logits.argmax(-1).astype(np.int32)
    out[key + "/dec_max"] = logits.max(-1)
    # cross attention weights (post-softmax) of the last layer, head 0
    ca = r.cross_attentions[-1][0, 0].numpy()  # [T, 1500]
    out[key + "/dec_xattn_l_last_h0_cols"] = np.arange(0, d.n_audio_ctx, 11).astype(np.int32)
    out[key + "/dec_xattn_l_last_h0"] = ca[:, ::11]


def gen_rules(out):
    from transformers.generation.logits_process import (SuppressTokensAtBeginLogitsProcessor,
                                                        SuppressTokensLogitsProcessor,
                                                        WhisperTimeStampLogitsProcessor)
    from transformers import GenerationConfig
    rng = np.random.default_rng(7)
    for V in (51865, 51866):
        sp = O.special_tokens(V)
        tb = sp.timestamp_begin
        histories = [[], [tb], [tb, 500], [tb, 500, tb + 40], [tb, 500, tb + 40, tb + 40], [tb + 3, 9, 10],
                     [1, 2, 3], [tb + 1499, 7, tb + 1500]]
        cfg = GenerationConfig(eos_token_id=sp.eot, bos_token_id=sp.eot)
        cfg.no_timestamps_token_id = sp.no_timestamps
        cfg.max_initial_timestamp_index = 50
        suppress = [1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93, 359]
        for i, hist in enumerate(histories):
            for variant in range(2):
                logits = rng.normal(0, 3, V).astype(np.float32)
                if variant == 1:  # make timestamps dominant to exercise the logsumexp rule
                    logits[tb:] += 4.0
                logits = logits.astype(np.float16).astype(np.float32)  # stored as f16: keep the fixture small
                prefix = [sp.sot, sp.lang0, sp.transcribe]
                ids = torch.tensor([prefix + hist])
                s = torch.from_numpy(logits.copy())[None]
                s = SuppressTokensAtBeginLogitsProcessor([220, sp.eot], len(prefix))(ids, s)
                s = SuppressTokensLogitsProcessor(suppress)(ids, s)
                s = WhisperTimeStampLogitsProcessor(cfg, begin_index=len(prefix))(ids, s)
                k = f"rules/{V}/{i}/{variant}"
                out[k + "/hist"] = np.array(hist if hist else [-1], np.int32)
                out[k + "/logits"] = logits.astype(np.float16)
                out[k + "/masked"] = np.packbits(np.isneginf(s[0].numpy()))
        out[f"rules/{V}/suppress"] = np.array(suppress, np.int32)


def gen_dtw(out):
    from transformers.models.whisper.generation_whisper import _dynamic_time_warping, _median_filter
    rng = np.random.default_rng(9)
    for i, (n, m) in enumerate([(5, 40), (12, 150), (1, 7), (30, 300)]):
        x = rng.normal(size=(n, m)).astype(np.float32)
        ti, tj = _dynamic_time_warping(x)
        out[f"dtw/{i}/x"] = x
        out[f"dtw/{i}/ti"] = np.asarray(ti, np.int32)
        out[f"dtw/{i}/tj"] = np.asarray(tj, np.int32)
    for i, (h, n, m) in enumerate([(4, 6, 50), (2, 9, 200)]):
        x = rng.normal(size=(h, n, m)).astype(np.float32)
        out[f"medfilt/{i}/x"] = x
        out[f"medfilt/{i}/y"] = _median_filter(torch.from_numpy(x), 7).numpy()


def main():
    torch.manual_seed(0)
    out = {}
    gen_logmel(out)
    gen_rules(out)
    gen_dtw(out)
    for name, seed, dtype in [("micro", 1, "bf16"), ("tiny", 2, "bf16"), ("tiny", 3, "f16")]:
        gen_model(out, name, seed, dtype)
    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


if __name__ == "__main__":
    main()
