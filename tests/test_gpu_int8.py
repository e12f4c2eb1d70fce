"""The CTranslate2 int8 grid on the GPU: model dtype WMX_DTYPE_I8, compute_type "int8_float16"
(the reference's 8-bit mode, 一键实时识别麦克风.py:304; int8 on its CPU path, asr_components.py:256-261).

Every decoder projection and the logits projection run on int8 weights with CTranslate2's per-row scales (the
packed8 layout of the fp8 decode, int8 bytes widened exactly to f16 in registers, the row's 1 / scale on the fp32
result); activations f16.

* A CT2 int8 directory at large-v3 width (model.bin written by wmx.ct2 from PRNG weights with CT2's int8 rule) loads
  with its own grid: the device's int8 bytes and row scales equal the file's, bit for bit, for every kept weight.
* Teacher-forced decode steps against oracle.int8_decoder_weights with the file's scales (q / scale in f32) on the
  device's own encoder output: the f16 step bound of tests/test_gpu_step.py (rel-L2 <= 5e-3, argmax equal wherever
  the oracle's margin exceeds twice the row's error) at the bench's per-group shape (4 windows x beam 5).
* A model initialised synthetically derives the scales by CT2's rule on device: bytes and scales equal
  oracle.int8_rows of its 16-bit weights.
* End to end through the drop-in adapter with compute_type "int8_float16".
Parity with CTranslate2's own int8 arithmetic (it also quantizes the activations of its GEMMs) is unpinned: the
engine is not installed here."""
import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

pytestmark = pytest.mark.gpu

WIDE2 = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 2)  # large-v3 width, 1 encoder layer, 2 decoder layers


def _dims(E, d):
    return E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                       d.n_text_head, d.n_text_layer)


def _kept(d):
    out = {"decoder.embed_tokens.weight": (d.n_vocab, d.n_text_state)}
    for i in range(d.n_text_layer):
        for n in O.FP8_DEC_LINEARS:
            rows = 4 * d.n_text_state if n == "fc1" else d.n_text_state
            cols = 4 * d.n_text_state if n == "fc2" else d.n_text_state
            out[f"decoder.layers.{i}.{n}.weight"] = (rows, cols)
    return out


@pytest.fixture(scope="module")
def ct2_int8(tmp_path_factory):
    from wmx import ct2
    from wmx import engine as E
    from wmx.transcribe import _load_checkpoint
    d = WIDE2
    W = O.make_weights(d, 7, "f16")
    v, al = ct2.hf_to_ct2(W, dict(n_audio_layer=d.n_audio_layer, n_text_layer=d.n_text_layer), "int8")
    path = tmp_path_factory.mktemp("ct2_int8")
    ct2.write_model_bin(str(path / "model.bin"), v, al)
    file_scales = {}
    _, deq = ct2.ct2_to_hf(ct2.resolve_aliases(v, al), file_scales)
    m = E.Model(_dims(E, d), 0, "int8_float16")
    assert m.int8
    _load_checkpoint(m, str(path))
    return m, deq, file_scales, W


def test_int8_checkpoint_keeps_its_exact_grid(ct2_int8):
    m, deq, file_scales, _ = ct2_int8
    n = 0
    for name, shape in _kept(WIDE2).items():
        q, sc = m.get_int8(name, shape)
        qf, sf = O.int8_rows(deq[name], file_scales[name])  # = the file's q (tests/test_ct2_format.py)
        np.testing.assert_array_equal(sc, file_scales[name], err_msg=name)
        np.testing.assert_array_equal(q, qf, err_msg=name)
        n += 1
    print("int8 weights on the checkpoint's grid:", n)


def test_int8_arena_copy_keeps_the_checkpoint_scales(ct2_int8):
    """The weight broadcast of a CT2 int8 checkpoint: a second model that receives the first one's
    parameter region (what share_weights broadcasts over RCCL; here one device-to-device copy) and derives its copies
    (wmx_model_arena_loaded) keeps the checkpoint's row scales and int8 bytes bit for bit -- the given / derived state
    of every scale row travels with the region, so no rank re-derives a scale the checkpoint gave."""
    import ctypes as C
    from wmx import engine as E
    m, deq, file_scales, _ = ct2_int8
    m2 = E.Model(_dims(E, WIDE2), 0, "int8_float16")
    (src, n1), (dst, n2) = m.arena(), m2.arena()
    assert n1 == n2
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(dst, src, n1, 3) == 0  # hipMemcpyDeviceToDevice
    assert hip.hipDeviceSynchronize() == 0
    m2.mark_loaded()
    for name, shape in _kept(WIDE2).items():
        q1, s1 = m.get_int8(name, shape)
        q2, s2 = m2.get_int8(name, shape)
        np.testing.assert_array_equal(s2, file_scales[name], err_msg=name)
        np.testing.assert_array_equal(s2, s1, err_msg=name)
        np.testing.assert_array_equal(q2, q1, err_msg=name)
    m2.close()


@pytest.mark.parametrize("B,K", [(4, 5), (20, 1)])
def test_int8_forced_decode_matches_oracle(ct2_int8, B, K):
    """The int8 rule the product runs (INTEGRATION.md 'The int8 arithmetic rule'): CTranslate2's int8 weight grid and
    row scales against 16-bit activation rows: the oracle's int8_decoder_weights dequantizes the weights and keeps
    the activations in the model's 16-bit type (CTranslate2's dynamic int8 activation rows are not restated)."""
    from wmx import engine as E
    import test_gpu_step as S
    m, deq, file_scales, W0 = ct2_int8
    d = WIDE2
    sp = O.special_tokens(d.n_vocab)
    W = {name: m.get_tensor(name, shape) for name, shape, _, _ in O.tensor_specs(d)}
    W["encoder.embed_positions.weight"] = O.sinusoids(1500, d.n_audio_state)
    Wi = O.int8_decoder_weights(W, d, file_scales)
    ctx = E.Context(m, max_batch=B, beam_size=K, max_new_tokens=64, word_timestamps=False)
    lens = [480000, 150000, 320000, 16000, 240000]
    mels = np.stack([O.logmel_segment(synth.speech_like(400 + i, lens[i % 5]), d.n_mels) for i in range(B)])
    encs = list(ctx.encode(mels))
    n = 16
    tok, par = S._forced_stream(np.random.default_rng(17 + B), n, B * K, K)
    prefix = [[sp.sot, sp.lang0, sp.transcribe]] * B
    top1, lg = ctx.forced_decode(prefix, tok, par, logits_every=1)
    ref_top1, ref_margin, ref_lg = O.forced_rows(Wi, d, encs, prefix, tok, par, K)
    S._check_forced(f"int8 decode B={B} K={K}", "f16", top1, lg, 1, ref_top1, ref_margin, ref_lg, 12)
    # the int8 grid is live: the decode of the weights before CT2 quantized them sits measurably away
    W0 = dict(W0)
    W0["encoder.embed_positions.weight"] = W["encoder.embed_positions.weight"]
    _, _, lg16 = O.forced_rows(W0, d, encs[:1], prefix[:1], tok[:2, :K], par[:2, :K], K)
    d16 = float(np.linalg.norm(lg[1, 0] - lg16[1][0]) / np.linalg.norm(lg16[1][0]))
    print("int8 decode vs the unquantized weights, row 0 step 1 rel_l2", d16)
    assert d16 > 5e-3, d16


def test_int8_synthetic_model_derives_ct2_scales():
    from wmx import engine as E
    d = O.Dims(80, 51865, 384, 6, 1, 384, 6, 2)
    m = E.Model(_dims(E, d), 0, "int8_float16").init_synthetic(3)
    for name, shape in list(_kept(d).items())[:6]:
        q, sc = m.get_int8(name, shape)
        qo, so = O.int8_rows(m.get_tensor(name, shape))
        np.testing.assert_array_equal(sc, so, err_msg=name)
        np.testing.assert_array_equal(q, qo, err_msg=name)


def test_int8_through_the_adapter():
    from wmx.asr import MI355XWhisperASR
    asr = MI355XWhisperASR(lan="auto", modelsize="micro", device="cuda", compute_type="int8_float16",
                           transcribe_kwargs={"beam_size": 5}, max_new_tokens=16)
    assert asr.model.model.int8
    segs = asr.transcribe(synth.speech_like(31, 16000 * 5))
    words = asr.ts_words(segs)
    assert isinstance(segs, list)
    for s, e, w in words:
        assert 0.0 <= s <= e <= 5.1
