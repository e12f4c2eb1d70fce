"""Silero VAD v5 on the GPU (csrc/wmx_vad.hip through wmx_vad_process) against the float64 oracle
(oracle/silero_np.py).  Parity unpinned against the Silero model itself (weights are torch.hub-only, reference
asr_components.py:96); the oracle is pinned to torch.nn's modules in tests/test_vad_oracle.py.

Tolerance: |p_gpu - p_oracle| <= 2e-5 per window (f32 accumulation over <= 387-term dot products and a 128-step
LSTM recursion per call, against float64).  The weights are the synthetic set with a gain of 5 so that the
probabilities spread over ~0.3 (PyTorch-default-scale random weights give a near-constant 0.515, which would not
test much).
"""
import numpy as np
import pytest

from oracle import silero_np as S

pytestmark = pytest.mark.gpu
TOL = 2e-5


def _weights(gain=5.0, seed=3):
    from wmx import vad
    W = vad.synthetic_state_dict(seed)
    return {k: (v if k == "stft.forward_basis_buffer" else (v * gain).astype(np.float32)) for k, v in W.items()}


def _audio(seed, n_win):
    from wmx import synth
    rng = np.random.default_rng(seed)
    a = synth.speech_like(seed, 512 * n_win) * np.repeat(rng.uniform(0.0, 1.5, n_win), 512)
    return a.astype(np.float32)


def test_multi_stream_multi_call_parity():
    from wmx import vad
    W = _weights()
    eng = vad.SileroVADEngine(W, max_streams=16, max_windows=8)
    ora = S.SileroStreams(W, 16)
    slots = [3, 0, 7, 12, 15, 1, 9, 4, 2, 11, 6, 14]
    audio = {s: _audio(100 + s, 1 + 3 + 2 + 8) for s in slots}
    pos = 0
    worst = 0.0
    for k in (1, 3, 2, 8):
        chunk = {s: audio[s][pos * 512:(pos + k) * 512] for s in slots}
        got = eng.process(chunk)
        ref = ora.process(slots, [chunk[s].astype(np.float64) for s in slots])
        for i, s in enumerate(slots):
            assert got[s].shape == (k,)
            worst = max(worst, float(np.max(np.abs(got[s] - ref[i]))))
        pos += k
        if k == 3:  # reset one slot mid-stream: its state and context restart from zeros
            eng.reset(7)
            ora.reset(7)
    print(f"vad parity: worst |dp| = {worst:.2e} over {len(slots)} streams x {pos} windows")
    assert worst <= TOL


def test_slot_subsets_do_not_disturb_other_slots():
    from wmx import vad
    W = _weights(seed=8)
    eng = vad.SileroVADEngine(W, max_streams=8, max_windows=4)
    ora = S.SileroStreams(W, 8)
    a = {s: _audio(200 + s, 8) for s in range(8)}
    for step in range(4):
        active = [s for s in range(8) if (s + step) % 3 != 0]
        chunk = {s: a[s][step * 1024:(step + 1) * 1024] for s in active}
        got = eng.process(chunk)
        ref = ora.process(active, [chunk[s].astype(np.float64) for s in active])
        for i, s in enumerate(active):
            np.testing.assert_allclose(got[s], ref[i], atol=TOL, rtol=0)


def test_full_node_batch_64_streams():
    """A tick of the streaming front end at config 4's shape (64 streams) with a backlog of 16 windows each."""
    from wmx import vad
    W = _weights(seed=5)
    eng = vad.SileroVADEngine(W, max_streams=64, max_windows=16)
    ora = S.SileroStreams(W, 64)
    slots = list(range(64))
    chunk = {s: _audio(300 + s, 16) for s in slots}
    got = eng.process(chunk)
    ref = ora.process(slots, [chunk[s].astype(np.float64) for s in slots])
    err = max(float(np.max(np.abs(got[s] - ref[i]))) for i, s in enumerate(slots))
    assert err <= TOL, err
    assert np.ptp(ref) > 0.05


def test_model_object_in_the_vad_iterator():
    """SileroVAD is the `model` of VADIterator / DynamicVADIterator (asr_components.py:23-34): the same events as the
    oracle-backed model on the same audio (windows whose probability is within 1e-4 of the threshold would be a
    legitimate f32 tie; none occur on this input)."""
    from wmx import online, vad
    W = _weights(seed=11)

    class OracleModel:
        def __init__(self):
            self.s = S.SileroStreams(W, 1)
            self.p = []

        def reset_states(self):
            self.s.reset(0)

        def __call__(self, x, sr=16000):
            p = float(self.s.process([0], [np.asarray(x, np.float64)])[0, 0])
            self.p.append(p)
            return p

    eng = vad.SileroVADEngine(W, max_streams=2, max_windows=2)
    om = OracleModel()
    audio = _audio(21, 80)
    thr = float(np.median([om(audio[i * 512:(i + 1) * 512]) for i in range(80)]))
    om.reset_states()
    om.p.clear()
    it_gpu = online.DynamicVADIterator(vad.SileroVAD(eng, slot=1), threshold=thr)
    it_ref = online.DynamicVADIterator(om, threshold=thr)
    ev_gpu = [it_gpu(audio[i:i + 640]) for i in range(0, len(audio), 640)]
    ev_ref = [it_ref(audio[i:i + 640]) for i in range(0, len(audio), 640)]
    assert min(abs(p - thr) for p in om.p) > 1e-4
    assert ev_gpu == ev_ref
    assert any(e is not None for e in ev_ref)


def test_stream_vad_batches_like_single_calls():
    from wmx import vad
    W = _weights(seed=13)
    eng_b = vad.SileroVADEngine(W, max_streams=8, max_windows=8)
    eng_s = vad.SileroVADEngine(W, max_streams=8, max_windows=8)
    sv = vad.StreamVAD(eng_b)
    rng = np.random.default_rng(1)
    audio = {s: _audio(400 + s, 12) for s in range(5)}
    pos = {s: 0 for s in audio}
    got = {s: [] for s in audio}
    for _ in range(10):
        feed = {}
        for s in audio:
            n = int(rng.integers(0, 1400))
            feed[s] = audio[s][pos[s]:pos[s] + n]
            pos[s] += len(feed[s])
        for s, p in sv.step(feed).items():
            got[s].extend(p.tolist())
    for s in audio:
        m = vad.SileroVAD(eng_s, slot=s)  # (constructing one resets the slot)
        single = [m(audio[s][i * 512:(i + 1) * 512]) for i in range(len(got[s]))]
        np.testing.assert_allclose(got[s], single, atol=1e-6, rtol=0)


def test_errors_are_reported():
    from wmx import _lib, vad
    W = _weights()
    eng = vad.SileroVADEngine(W, max_streams=4, max_windows=2)
    with pytest.raises(ValueError):
        eng.process({0: np.zeros(500, np.float32)})
    with pytest.raises(_lib.WmxError):
        eng.process({0: np.zeros(512 * 3, np.float32)})  # more windows than max_windows
    with pytest.raises(ValueError):
        vad.SileroVAD(eng, slot=0)(np.zeros(256, np.float32))
    import ctypes as C
    h = C.c_void_p()
    _lib.check(_lib.lib.wmx_vad_create(0, 2, 2, C.byref(h)))
    x = np.zeros(512, np.float32)
    p = np.zeros(1, np.float32)
    s = np.array([0], np.int32)
    assert _lib.lib.wmx_vad_process(h, _lib.fptr(x), 512, _lib.iptr(s), 1, 1, _lib.fptr(p)) != 0  # no weights
    assert b"not fully loaded" in _lib.lib.wmx_last_error()
    dup = np.array([1, 1], np.int32)
    _lib.lib.wmx_vad_free(h)
    with pytest.raises(_lib.WmxError):
        _lib.check(_lib.lib.wmx_vad_process(eng._h, _lib.fptr(np.zeros(1024, np.float32)), 512, _lib.iptr(dup), 2, 1,
                                            _lib.fptr(np.zeros(2, np.float32))))


def test_checkpoint_path_through_the_vac_processor(tmp_path):
    """A Silero v5 safetensors file (with the TorchScript `_model.` prefix) selected by path in
    DynamicVACOnlineASRProcessor(vad_model=...) gives the oracle's probabilities on those weights."""
    from safetensors.numpy import save_file

    from wmx import online, vad
    W = _weights(seed=17)
    p = str(tmp_path / "silero_v5.safetensors")
    save_file({"_model." + k: np.ascontiguousarray(v) for k, v in W.items()}, p)
    m = vad.silero_model(p)
    ora = S.SileroStreams(W, 1)
    a = _audio(31, 6)
    got = [m(a[i * 512:(i + 1) * 512]) for i in range(6)]
    np.testing.assert_allclose(got, ora.process([0], [a.astype(np.float64)])[0], atol=TOL, rtol=0)

    class NullASR:
        sep = ""

    proc = online.DynamicVACOnlineASRProcessor(1.0, NullASR(), vad_model=p)
    assert isinstance(proc.vac.vad.model, vad.SileroVAD)


def test_use_vad_through_the_adapter():
    """CustomFasterWhisperASR.use_vad() (asr_components.py:307-309) turns on faster-whisper's vad_filter: the device
    Silero network scores the buffer, only speech chunks are transcribed, times map back to the buffer.  With the
    synthetic weights the network scores everything as speech at the default threshold, so the chunk is the whole
    buffer; the speech-chunk logic itself is pinned by the host tests (tests/test_host_transcribe.py)."""
    from wmx import synth, vad
    from wmx.asr import MI355XWhisperASR
    asr = MI355XWhisperASR(lan="auto", modelsize="micro", device="cuda", compute_type="float16",
                           transcribe_kwargs={"beam_size": 1}, max_new_tokens=16)
    audio = synth.speech_like(61, 16000 * 6)
    base = asr.transcribe(audio)
    asr.use_vad()
    assert asr.transcribe_kargs.get("vad_filter") is True
    probs = vad.speech_probs(asr.model.vad_engine(), audio)
    chunks = vad.get_speech_timestamps(probs, len(audio))
    segs = asr.transcribe(audio)
    dur = len(audio) / 16000
    assert all(0.0 <= s.start <= s.end <= dur + 0.02 for s in segs)
    if chunks == [{"start": 0, "end": len(audio)}]:
        assert [(s.start, s.end, s.text) for s in segs] == [(s.start, s.end, s.text) for s in base]
