"""CPU restatement of the Silero VAD v5 network, 16 kHz branch — TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py): the product path is wmx.vad + csrc/wmx_vad.hip.

The reference loads the network at run time with torch.hub (asr_components.py:96,
`torch.hub.load(repo_or_dir='snakers4/silero-vad', model='silero_vad')`) and calls it once per 512-sample window
through whisper_streaming's VADIterator (`speech_prob = self.model(x, self.sampling_rate).item()`; reached from
DynamicVADIterator.__call__, asr_components.py:58-78).  Neither the weights nor the TorchScript code are in the
reference or in this image, so this file restates the published v5 architecture (silero-vad 5.x, the model the hub
call returns):

* wrapper: the 512 new samples are prefixed with the last 64 samples of the previous call's input (zeros after
  reset_states); the LSTM state (h, c) carries across calls;
* STFT as a strided conv: ReflectionPad1d((0, 64)) of the 576-sample input, conv1d with a [258, 1, 256] basis
  (129 real rows, 129 imaginary rows; stride 128 -> 4 frames), magnitude sqrt(re^2 + im^2) -> [129, 4];
* encoder: 4 x (Conv1d(k=3, padding=1) -> ReLU) with channels 129->128 (stride 1), 128->64 (2), 64->64 (2),
  64->128 (1) -> [128, 1];
* decoder: LSTMCell(128, 128) (torch gate order i, f, g, o), then ReLU -> Conv1d(128, 1, 1) -> Sigmoid; the
  probability is the mean over the single remaining frame.

Parity unpinned against the Silero model itself (no weights, no code here).  What is pinned: the torch-op semantics
this restatement relies on (reflection padding, conv stride / padding, LSTMCell gate order) against torch.nn's own
modules on the same weights (tests/test_vad_oracle.py).  Arithmetic in float64.
"""
from __future__ import annotations

import numpy as np

WINDOW, CONTEXT, NFFT, HOP, HIDDEN = 512, 64, 256, 128, 128
ENCODER = ((129, 128, 1), (128, 64, 2), (64, 64, 2), (64, 128, 1))  # (in, out, stride), kernel 3, padding 1


def tensor_shapes():
    """Silero v5 state-dict names (16 kHz branch, without the `_model.` prefix) -> shapes."""
    s = {"stft.forward_basis_buffer": (2 * (NFFT // 2 + 1), 1, NFFT)}
    for i, (ci, co, _) in enumerate(ENCODER):
        s[f"encoder.{i}.reparam_conv.weight"] = (co, ci, 3)
        s[f"encoder.{i}.reparam_conv.bias"] = (co,)
    s["decoder.rnn.weight_ih"] = (4 * HIDDEN, HIDDEN)
    s["decoder.rnn.weight_hh"] = (4 * HIDDEN, HIDDEN)
    s["decoder.rnn.bias_ih"] = (4 * HIDDEN,)
    s["decoder.rnn.bias_hh"] = (4 * HIDDEN,)
    s["decoder.decoder.2.weight"] = (1, HIDDEN, 1)
    s["decoder.decoder.2.bias"] = (1,)
    return s


def reflect_pad_right(x, n=CONTEXT):
    """torch.nn.ReflectionPad1d((0, n)) on the last axis: x[L-2], x[L-3], ... (the edge sample is not repeated)."""
    L = x.shape[-1]
    return np.concatenate([x, x[..., L - 2:L - 2 - n:-1]], axis=-1)


def stft_magnitude(W, x576):
    """[N, 576] -> [N, 129, 4]."""
    basis = np.asarray(W["stft.forward_basis_buffer"], np.float64)[:, 0, :]  # [258, 256]
    xp = reflect_pad_right(np.asarray(x576, np.float64))  # [N, 640]
    nfr = (xp.shape[-1] - NFFT) // HOP + 1
    frames = np.stack([xp[:, t * HOP:t * HOP + NFFT] for t in range(nfr)], axis=1)  # [N, 4, 256]
    out = np.einsum("ntk,ck->nct", frames, basis)  # [N, 258, 4]
    c = NFFT // 2 + 1
    return np.sqrt(out[:, :c] ** 2 + out[:, c:] ** 2)


def conv1d_k3(x, w, b, stride):
    """torch.nn.functional.conv1d(x, w, b, stride=stride, padding=1), x [N, Cin, L], w [Cout, Cin, 3]."""
    N, Cin, L = x.shape
    Lout = (L + 2 - 3) // stride + 1
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1)))
    cols = np.stack([xp[:, :, t * stride:t * stride + 3] for t in range(Lout)], axis=1)  # [N, Lout, Cin, 3]
    return np.einsum("ntik,oik->not", cols, np.asarray(w, np.float64)) + np.asarray(b, np.float64)[None, :, None]


def encode(W, x576):
    """The context-free part of one window (STFT + encoder), batched over windows: [N, 576] -> [N, 128]."""
    h = stft_magnitude(W, x576)
    for i, (_, _, stride) in enumerate(ENCODER):
        h = np.maximum(conv1d_k3(h, W[f"encoder.{i}.reparam_conv.weight"], W[f"encoder.{i}.reparam_conv.bias"],
                                 stride), 0.0)
    assert h.shape[-1] == 1
    return h[:, :, 0]


def _sigmoid(v):
    return 1.0 / (1.0 + np.exp(-v))


def lstm_cell(W, x, h, c):
    """torch.nn.LSTMCell: gates = x W_ih^T + b_ih + h W_hh^T + b_hh, chunked (i, f, g, o)."""
    g = (x @ np.asarray(W["decoder.rnn.weight_ih"], np.float64).T + np.asarray(W["decoder.rnn.bias_ih"], np.float64)
         + h @ np.asarray(W["decoder.rnn.weight_hh"], np.float64).T + np.asarray(W["decoder.rnn.bias_hh"], np.float64))
    i, f, gg, o = np.split(g, 4, axis=-1)
    c2 = _sigmoid(f) * c + _sigmoid(i) * np.tanh(gg)
    return _sigmoid(o) * np.tanh(c2), c2


def decode_prob(W, h):
    """ReLU -> Conv1d(128, 1, 1) -> Sigmoid on the LSTM output; the mean over the one frame is the frame."""
    w2 = np.asarray(W["decoder.decoder.2.weight"], np.float64)[0, :, 0]
    b2 = float(np.asarray(W["decoder.decoder.2.bias"], np.float64)[0])
    return _sigmoid(np.maximum(h, 0.0) @ w2 + b2)


class SileroStreams:
    """The v5 wrapper's per-call semantics for S independent streams: context prefix, carried (h, c)."""

    def __init__(self, W, n_streams):
        self.W = W
        self.ctx = np.zeros((n_streams, CONTEXT))
        self.h = np.zeros((n_streams, HIDDEN))
        self.c = np.zeros((n_streams, HIDDEN))

    def reset(self, s=None):
        sl = slice(None) if s is None else slice(s, s + 1)
        self.ctx[sl] = 0.0
        self.h[sl] = 0.0
        self.c[sl] = 0.0

    def process(self, streams, pcm):
        """pcm [len(streams)][k * 512] (k >= 1 windows per stream, processed in order) -> probs [len, k]."""
        pcm = np.asarray(pcm, np.float64)
        S, n = pcm.shape
        assert n % WINDOW == 0 and n > 0
        k = n // WINDOW
        full = np.concatenate([self.ctx[list(streams)], pcm], axis=1)  # [S, 64 + k * 512]
        x576 = np.stack([full[:, j * WINDOW:j * WINDOW + WINDOW + CONTEXT] for j in range(k)], axis=1)
        enc = encode(self.W, x576.reshape(S * k, -1)).reshape(S, k, HIDDEN)
        probs = np.empty((S, k))
        for si, s in enumerate(streams):
            h, c = self.h[s], self.c[s]
            for j in range(k):
                h, c = lstm_cell(self.W, enc[si, j], h, c)
                probs[si, j] = decode_prob(self.W, h)
            self.h[s], self.c[s] = h, c
            self.ctx[s] = full[si, -CONTEXT:]
        return probs
