"""The stream-K remainder of the persistent 256² encoder GEMM (G256Sk, wmx_gemm.hip gemm256_kernel): with T tiles
on a grid of G = 256 workgroups, the last T mod G tiles are split over K across all workgroups; contributors store
partial accumulator images, take tickets, and the last one sums the parts in k order and runs the epilogue.

At large-v3 width with 8 windows (12000 rows) every encoder GEMM of the bench takes that path: qkv (705 tiles, 193
split), out-projection and fc2 (235 tiles, all split over 256 workgroups), fc1 (940, 172 split), conv2 (235 split)
and the cross-K/V GEMM.  Checked:
  * the encoder output against the oracle (relative L2 <= 3e-2, the bf16 bound of tests/test_gpu_parity.py);
  * bit-exact across repeated calls (the ticket order varies from run to run; the k-order sum must not);
  * against the same encoder with the split turned off (WMX_G256_SK=0, a child process): only the summation order
    differs, so the distance must stay at the level of one bf16 rounding of the outputs (relative L2 <= 5e-3).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import whisper_np as O
from wmx import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WIDE1 = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 1)
CHILD = r"""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.environ["WMX_ROOT"], "realtime-whisper-asr_amd"), os.environ["WMX_ROOT"]]
from wmx import engine as E
from oracle import whisper_np as O
from wmx import synth
d = O.Dims(128, 51866, 1280, 20, 1, 1280, 20, 1)
m = E.Model(E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                        d.n_text_head, d.n_text_layer), 0, "bfloat16").init_synthetic(31)
mels = np.stack([O.logmel_segment(synth.speech_like(1300 + i, 480000 - 37000 * i), 128) for i in range(8)])
ctx = E.Context(m, max_batch=8, beam_size=1, max_new_tokens=8, word_timestamps=False)
np.save(sys.argv[1], ctx.encode(mels))
"""


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _child(path, sk):
    env = dict(os.environ, WMX_ROOT=ROOT)
    env["WMX_G256_SK"] = "1" if sk else "0"
    r = subprocess.run([sys.executable, "-c", CHILD, path], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return np.load(path)


def test_streamk_encoder_oracle_determinism_and_split_off(tmp_path):
    from wmx import engine as E
    d = WIDE1
    m = E.Model(E.ModelDims(d.n_mels, d.n_vocab, d.n_audio_state, d.n_audio_head, d.n_audio_layer, d.n_text_state,
                            d.n_text_head, d.n_text_layer), 0, "bfloat16").init_synthetic(31)
    mels = np.stack([O.logmel_segment(synth.speech_like(1300 + i, 480000 - 37000 * i), 128) for i in range(8)])
    ctx = E.Context(m, max_batch=8, beam_size=1, max_new_tokens=8, word_timestamps=False)
    a = ctx.encode(mels)
    for _ in range(2):
        np.testing.assert_array_equal(ctx.encode(mels), a)
    W = O.make_weights(d, 31, "bf16")
    for b in (0, 5, 7):
        e = rel_l2(a[b], O.encoder(W, d, mels[b]))
        print(f"window {b}: encoder rel_l2 vs oracle {e:.2e}")
        assert e <= 3e-2, (b, e)
    on = _child(str(tmp_path / "on.npy"), True)
    off = _child(str(tmp_path / "off.npy"), False)
    np.testing.assert_array_equal(on, a)  # a fresh process, same split: same bits
    e = rel_l2(on, off)
    print(f"split vs unsplit encoder rel_l2 {e:.2e}")
    assert e <= 5e-3, e
