"""Checkpoint ingestion: HF-named safetensors -> wmx_model_set_tensor, bit-exact.

The build-owned PRNG weights are written as a HF Whisper state dict ("model." prefix, tied proj_out) in f32 and in
bf16 storage, loaded through wmx.transcribe._load_checkpoint into a fresh model, and every tensor must read back
bit-identical to init_synthetic's (the set path rounds to the model dtype and packs the decoder projections;
get_tensor unpacks).  The loaded model must then transcribe token-identically to the synthetic one."""
import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("storage", ["f32", "bf16"])
def test_safetensors_roundtrip_bit_exact(tmp_path, storage):
    import torch
    from safetensors.torch import save_file

    from wmx import engine as E
    from wmx.transcribe import _load_checkpoint
    d = O.DIMS["micro"]
    ref = E.Model("micro", 0, "bfloat16").init_synthetic(3)
    sd = {}
    for name, shape, _, _ in O.tensor_specs(d):
        sd["model." + name] = torch.from_numpy(ref.get_tensor(name, shape).copy())
    sd["model.encoder.embed_positions.weight"] = torch.from_numpy(
        ref.get_tensor("encoder.embed_positions.weight", (1500, d.n_audio_state)).copy())
    sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
    if storage == "bf16":
        sd = {k: v.to(torch.bfloat16) for k, v in sd.items()}
    sd = {k: v.contiguous().clone() for k, v in sd.items()}
    save_file(sd, str(tmp_path / "model.safetensors"))
    m = E.Model("micro", 0, "bfloat16")
    _load_checkpoint(m, str(tmp_path))
    n = 0
    for name, shape, _, _ in O.tensor_specs(d):
        np.testing.assert_array_equal(m.get_tensor(name, shape), ref.get_tensor(name, shape), err_msg=name)
        n += 1
    assert n == len(O.tensor_specs(d))
    a = [synth.speech_like(91, 80000), synth.speech_like(92, 200000)]
    c1 = E.Context(ref, max_batch=2, beam_size=2, max_new_tokens=12, word_timestamps=False)
    c2 = E.Context(m, max_batch=2, beam_size=2, max_new_tokens=12, word_timestamps=False)
    r1, r2 = c1.transcribe(a), c2.transcribe(a)
    assert [r.tokens for r in r1] == [r.tokens for r in r2]
    print(storage, "tensors", n, "tokens", [len(r.tokens) for r in r1])


@pytest.mark.parametrize("q", ["float16", "int8"])
def test_ct2_model_dir(tmp_path, q):
    """A CTranslate2 directory (model.bin in the Whisper spec layout, as the reference's models_fast/ holds) written
    from the synthetic weights loads through _load_checkpoint: float16 storage reads back to the bf16 model
    bit-exactly wherever f16 holds the bf16 value, and transcribes like the synthetic model; int8 (per-row
    scales) is within its quantisation step."""
    from wmx import ct2
    from wmx import engine as E
    from wmx.transcribe import _load_checkpoint
    d = O.DIMS["micro"]
    ref = E.Model("micro", 0, "bfloat16").init_synthetic(3)
    sd = {name: ref.get_tensor(name, shape) for name, shape, _, _ in O.tensor_specs(d)}
    sd["encoder.embed_positions.weight"] = ref.get_tensor("encoder.embed_positions.weight", (1500, d.n_audio_state))
    v, al = ct2.hf_to_ct2(sd, dict(n_audio_layer=d.n_audio_layer, n_text_layer=d.n_text_layer), q)
    ct2.write_model_bin(str(tmp_path / "model.bin"), v, al)
    m = E.Model("micro", 0, "bfloat16")
    _load_checkpoint(m, str(tmp_path))
    worst = 0.0
    for name, shape, _, _ in O.tensor_specs(d):
        a, b = m.get_tensor(name, shape), sd[name]
        worst = max(worst, float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b))))))
    print(q, "worst relative tensor error", worst)
    assert worst <= (1e-2 if q == "float16" else 2e-2)
    a = [synth.speech_like(91, 80000), synth.speech_like(92, 200000)]
    r1 = E.Context(ref, max_batch=2, beam_size=2, max_new_tokens=12, word_timestamps=False).transcribe(a)
    r2 = E.Context(m, max_batch=2, beam_size=2, max_new_tokens=12, word_timestamps=False).transcribe(a)
    if q == "float16":
        assert [r.tokens for r in r1] == [r.tokens for r in r2]
    assert all(len(r.tokens) > 0 for r in r2)
