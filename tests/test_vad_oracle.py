"""Silero VAD restatement (oracle/silero_np.py) against torch.nn's own modules, and the VAD host plumbing (CPU).

Parity unpinned against the Silero model itself: its weights and TorchScript code are fetched by torch.hub at run
time (reference asr_components.py:96) and are not in the reference or this image.  What this file pins is the
restatement's use of torch op semantics: ReflectionPad1d((0, 64)), Conv1d(k=3, padding=1, stride), LSTMCell gate
order (i, f, g, o) and the v5 wrapper's 64-sample context / carried state, on the same weights, in float64.
"""
import numpy as np
import pytest
import torch

from oracle import silero_np as S


def _weights(gain=5.0):
    from wmx import vad
    W = vad.synthetic_state_dict(3)
    return {k: (v if k == "stft.forward_basis_buffer" else v * gain) for k, v in W.items()}


class TorchSilero(torch.nn.Module):
    """The v5 16 kHz graph from torch.nn modules (the architecture oracle/silero_np.py restates)."""

    def __init__(self, W):
        super().__init__()
        t = lambda a: torch.tensor(np.asarray(a, np.float64))
        self.pad = torch.nn.ReflectionPad1d((0, 64))
        self.basis = t(W["stft.forward_basis_buffer"])
        convs = []
        for i, (ci, co, s) in enumerate(S.ENCODER):
            c = torch.nn.Conv1d(ci, co, 3, stride=s, padding=1).double()
            c.weight.data = t(W[f"encoder.{i}.reparam_conv.weight"])
            c.bias.data = t(W[f"encoder.{i}.reparam_conv.bias"])
            convs += [c, torch.nn.ReLU()]
        self.encoder = torch.nn.Sequential(*convs)
        self.rnn = torch.nn.LSTMCell(128, 128).double()
        for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
            getattr(self.rnn, n).data = t(W[f"decoder.rnn.{n}"])
        self.out = torch.nn.Conv1d(128, 1, 1).double()
        self.out.weight.data = t(W["decoder.decoder.2.weight"])
        self.out.bias.data = t(W["decoder.decoder.2.bias"])
        self.reset_states()

    def reset_states(self):
        self.ctx = torch.zeros(1, 64, dtype=torch.float64)
        self.state = None

    @torch.no_grad()
    def forward(self, x):
        x = torch.cat([self.ctx, torch.tensor(np.asarray(x, np.float64))[None]], 1)  # [1, 576]
        self.ctx = x[:, -64:]
        f = torch.nn.functional.conv1d(self.pad(x[:, None, :]), self.basis, stride=128)
        mag = torch.sqrt(f[:, :129] ** 2 + f[:, 129:] ** 2)
        e = self.encoder(mag).squeeze(-1)
        h, c = self.rnn(e, self.state) if self.state is not None else self.rnn(e)
        self.state = (h, c)
        return float(torch.sigmoid(self.out(torch.relu(h)[..., None])).mean())


def test_shapes_match_product_names():
    from wmx import vad
    assert vad.tensor_shapes() == S.tensor_shapes()
    W = vad.synthetic_state_dict(0)
    assert {k: v.shape for k, v in W.items()} == S.tensor_shapes()
    assert all(v.dtype == np.float32 for v in W.values())


def test_reflection_pad_matches_torch():
    x = np.arange(576, dtype=np.float64)[None]
    ref = torch.nn.ReflectionPad1d((0, 64))(torch.tensor(x)[:, None])[:, 0].numpy()
    np.testing.assert_array_equal(S.reflect_pad_right(x), ref)


def test_stft_basis_is_a_windowed_dft():
    from wmx import vad
    B = vad.stft_basis()[:, 0, :].astype(np.float64)
    n = np.arange(256)
    tone = np.cos(2 * np.pi * 20 * n / 256)
    spec = np.hypot(B[:129] @ tone, B[129:] @ tone)
    assert int(np.argmax(spec)) == 20
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / 256)
    np.testing.assert_allclose(B[0], win, atol=1e-6)  # bin 0 real row = the window


def test_oracle_matches_torch_modules_over_a_stream():
    from wmx import synth
    W = _weights()
    tm = TorchSilero(W)
    st = S.SileroStreams(W, 2)
    rng = np.random.default_rng(0)
    audio = synth.speech_like(5, 512 * 24) * np.repeat(rng.uniform(0, 1, 24), 512)
    ref = [tm(audio[i * 512:(i + 1) * 512]) for i in range(24)]
    # the oracle in three calls of 1, 15 and 8 windows: context / state carry across calls
    got = np.concatenate([st.process([1], [audio[:512]])[0], st.process([1], [audio[512:512 * 16]])[0],
                          st.process([1], [audio[512 * 16:]])[0]])
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)
    assert np.ptp(ref) > 0.05  # the stress weights make the probabilities move
    tm.reset_states()
    st.reset(1)
    np.testing.assert_allclose(st.process([1], [audio[:1024]])[0], [tm(audio[:512]), tm(audio[512:1024])], atol=1e-12)


def test_vad_iterator_on_the_oracle_model():
    """The oracle model drives the VADIterator rules (wmx.online) like the Silero model does: events at window
    granularity, ends after min_silence."""
    from wmx import online, synth

    class OracleModel:
        def __init__(self, W):
            self.s = S.SileroStreams(W, 1)

        def reset_states(self):
            self.s.reset(0)

        def __call__(self, x, sr=16000):
            return float(self.s.process([0], [x])[0, 0])

    W = _weights()
    it = online.DynamicVADIterator(OracleModel(W), threshold=0.6)
    audio = synth.speech_like(9, 512 * 60)
    events = [it(audio[i:i + 640]) for i in range(0, len(audio), 640)]
    assert all(e is None or set(e) <= {"start", "end"} for e in events)


def test_vad_create_fails_cleanly_without_gpu():
    import ctypes as C

    from wmx import _lib
    if _lib.lib.wmx_device_count() > 0:
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    assert _lib.lib.wmx_vad_create(0, 4, 4, C.byref(h)) != 0
    assert _lib.lib.wmx_last_error()


def test_safetensors_loader_accepts_the_v5_prefix(tmp_path):
    from safetensors.numpy import save_file

    from wmx import vad
    W = _weights()
    p = str(tmp_path / "silero_v5.safetensors")
    save_file({"_model." + k: np.ascontiguousarray(v) for k, v in W.items()}, p)
    got = vad.load_state_dict(p)
    assert set(got) == set(W)
    for k in W:
        np.testing.assert_array_equal(got[k], W[k])
    save_file({k: np.ascontiguousarray(v) for k, v in W.items() if k != "decoder.rnn.bias_hh"}, p)
    with pytest.raises(KeyError):
        vad.load_state_dict(p)
