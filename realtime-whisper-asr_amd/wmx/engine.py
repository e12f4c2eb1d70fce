"""Thin Python handle over libwmx.so: a model (weight arena on one GPU) and decoding contexts.

This is plumbing for the drop-in ASR adapter (wmx.asr) and the benchmark; all arithmetic runs in the HIP
library.  Model dimensions follow openai-whisper ModelDimensions (what faster-whisper/CT2 checkpoints carry).
"""
from __future__ import annotations

import ctypes as C
import warnings
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from ._lib import check, fptr, iptr, lptr, lib


@dataclass(frozen=True)
class ModelDims:
    n_mels: int
    n_vocab: int
    n_audio_state: int
    n_audio_head: int
    n_audio_layer: int
    n_text_state: int
    n_text_head: int
    n_text_layer: int
    n_audio_ctx: int = 1500
    n_text_ctx: int = 448


MODEL_DIMS = {
    "tiny": ModelDims(80, 51865, 384, 6, 4, 384, 6, 4),
    "base": ModelDims(80, 51865, 512, 8, 6, 512, 8, 6),
    "small": ModelDims(80, 51865, 768, 12, 12, 768, 12, 12),
    "medium": ModelDims(80, 51865, 1024, 16, 24, 1024, 16, 24),
    "large-v2": ModelDims(80, 51865, 1280, 20, 32, 1280, 20, 32),
    "large-v3": ModelDims(128, 51866, 1280, 20, 32, 1280, 20, 32),
    "large-v3-turbo": ModelDims(128, 51866, 1280, 20, 32, 1280, 20, 4),
    "micro": ModelDims(80, 51865, 128, 2, 2, 128, 2, 2),
}
MODEL_DIMS["tiny.en"] = MODEL_DIMS["tiny"]
MODEL_DIMS["base.en"] = MODEL_DIMS["base"]
MODEL_DIMS["large"] = MODEL_DIMS["large-v3"]

# alignment heads of released checkpoints as (layer, head): the generation_config.json "alignment_heads" of the
# HF openai/whisper-large-v3 repo (not reachable offline; only used as the head set, any set is valid)
ALIGNMENT_HEADS = {
    "large-v3": [(7, 0), (10, 17), (12, 18), (13, 12), (16, 1), (17, 14), (19, 11), (21, 4), (24, 1), (25, 6)],
}


def _dims_struct(d: ModelDims) -> L.Dims:
    return L.Dims(d.n_mels, d.n_vocab, d.n_audio_ctx, d.n_audio_state, d.n_audio_head, d.n_audio_layer,
                  d.n_text_ctx, d.n_text_state, d.n_text_head, d.n_text_layer)


class Model:
    """Weights of one Whisper model resident in HBM of `device` (one arena)."""

    def __init__(self, name_or_dims="large-v3", device: int = 0, compute_type: str = "bfloat16"):
        self.dims = MODEL_DIMS[name_or_dims] if isinstance(name_or_dims, str) else name_or_dims
        self.name = name_or_dims if isinstance(name_or_dims, str) else "custom"
        ct = compute_type.lower()
        self.compute_type = ct
        if ct in ("bfloat16", "bf16"):
            self.dtype = L.WMX_DTYPE_BF16
        elif ct in ("float16", "f16", "fp16", "default", "auto"):
            self.dtype = L.WMX_DTYPE_F16
        elif ct in ("float8", "fp8", "mxfp8", "mx8", "float8_bfloat16"):
            # BASELINE config 5: encoder projections on the CDNA4 MX-fp8 MFMA, the decode on 8-bit weights and fp8
            # cross-K/V images (include/wmx.h WMX_DTYPE_MX8), activations bf16
            self.dtype = L.WMX_DTYPE_MX8
        elif ct in ("int8_float16", "int8", "int8_float32"):
            # CTranslate2's int8 modes (the reference's int8_float16, 一键实时识别麦克风.py:304; int8 on the CPU path,
            # asr_components.py:256-261): CT2's int8 grid -- int8 weights with CT2's per-row scales for every decoder
            # projection and the logits projection (include/wmx.h WMX_DTYPE_I8), f16 activations ("int8" /
            # "int8_float32" run them in f16 too: CT2 computes those in f32)
            self.dtype = L.WMX_DTYPE_I8
        elif ct == "int8_bfloat16":
            self.dtype = L.WMX_DTYPE_I8_BF16
        else:
            raise ValueError(f"compute_type {compute_type!r} is not supported on MI355X "
                             "(use float16 / bfloat16 / float8 / int8_float16)")
        self.device = device
        h = C.c_void_p()
        ds = _dims_struct(self.dims)
        check(lib.wmx_model_create(C.byref(ds), device, self.dtype, C.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def init_synthetic(self, seed: int) -> "Model":
        check(lib.wmx_model_init_synthetic(self._h, C.c_uint64(seed)))
        return self

    def set_tensor(self, name: str, value: np.ndarray):
        v = np.ascontiguousarray(value, dtype=np.float32)
        check(lib.wmx_model_set_tensor(self._h, name.encode(), fptr(v), v.size))

    def get_tensor(self, name: str, shape) -> np.ndarray:
        out = np.empty(shape, np.float32)
        check(lib.wmx_model_get_tensor(self._h, name.encode(), fptr(out), out.size))
        return out

    @property
    def int8(self) -> bool:
        """The CTranslate2 int8 grid (compute_type int8_float16 / int8 / int8_bfloat16)."""
        return self.dtype in (L.WMX_DTYPE_I8, L.WMX_DTYPE_I8_BF16)

    def set_row_scales(self, name: str, scale: np.ndarray):
        """int8 model: a decoder projection's (or the token embedding's) CT2 row scales, after its weight."""
        v = np.ascontiguousarray(scale, dtype=np.float32).reshape(-1)
        check(lib.wmx_model_set_row_scales(self._h, name.encode(), fptr(v), v.size))

    def get_int8(self, name: str, shape):
        """int8 model: (q int8 [rows][cols], CT2 scales [rows]) of one decoder projection as the device holds them."""
        q = np.empty(shape, np.int8)
        sc = np.empty(shape[0], np.float32)
        check(lib.wmx_model_get_int8(self._h, name.encode(), q.ctypes.data_as(C.POINTER(C.c_int8)), fptr(sc),
                                     shape[0], shape[1]))
        return q, sc

    def load_state_dict(self, sd: dict, row_scales: dict | None = None):
        """HF/openai-named fp32 tensors (a converted checkpoint); strips a leading 'model.'.  row_scales: a CT2 int8
        checkpoint's per-row scales by weight name (int8 models keep the checkpoint's exact int8 grid; other models
        ignore them -- the weights are the dequantized q / scale either way)."""
        for k, v in sd.items():
            k = k[6:] if k.startswith("model.") else k
            if k == "proj_out.weight":
                continue
            self.set_tensor(k, np.asarray(v, dtype=np.float32))
        if row_scales and self.int8:
            for k, v in row_scales.items():
                self.set_row_scales(k, v)
        check(lib.wmx_model_arena_loaded(self._h))

    def n_params(self) -> int:
        return int(lib.wmx_model_n_params(self._h))

    def arena(self):
        p, n = C.c_void_p(), C.c_size_t()
        check(lib.wmx_model_arena(self._h, C.byref(p), C.byref(n)))
        return p.value, n.value

    def mark_loaded(self):
        check(lib.wmx_model_arena_loaded(self._h))

    def close(self):
        if getattr(self, "_h", None):
            lib.wmx_model_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class WindowResult:
    tokens: list
    language: int
    language_prob: float
    sum_logprob: float
    avg_logprob: float
    no_speech_prob: float
    seek_frames: int
    jump_times: np.ndarray | None
    text_token_probs: np.ndarray | None


class Context:
    """Decoding context: batch capacity, beam, rules; owns device buffers and the decode-step hipGraph."""

    def __init__(self, model: Model, max_batch: int = 1, beam_size: int = 5, patience: float = 1.0,
                 length_penalty: float = 1.0, max_new_tokens: int = 448, task: str = "transcribe",
                 language: int | None = None, without_timestamps: bool = False,
                 max_initial_timestamp_index: int | None = 50, suppress_blank: bool = True,
                 suppress_tokens=(), word_timestamps: bool = True, alignment_heads=None,
                 median_filter_width: int = 7, use_graph: bool = True, max_audio_samples: int = 480000,
                 temperature: float = 0.0, best_of: int = 5, sample_seed: int = 0):
        self.model = model
        o = L.Opts()
        lib.wmx_opts_default(C.byref(o))
        o.max_batch = max_batch
        o.beam_size = beam_size
        o.patience = patience
        o.length_penalty = length_penalty
        o.max_new_tokens = max_new_tokens
        o.task = L.WMX_TASK_TRANSLATE if task == "translate" else L.WMX_TASK_TRANSCRIBE
        o.language = -1 if language is None else int(language)
        o.without_timestamps = int(without_timestamps)
        o.max_initial_timestamp_index = -1 if max_initial_timestamp_index is None else int(max_initial_timestamp_index)
        o.suppress_blank = int(suppress_blank)
        self._sup = np.ascontiguousarray(np.asarray(list(suppress_tokens), dtype=np.int32))
        o.suppress_tokens = iptr(self._sup) if self._sup.size else None
        o.n_suppress_tokens = int(self._sup.size)
        o.word_timestamps = int(word_timestamps)
        if alignment_heads:
            self._ah = np.ascontiguousarray(np.asarray(alignment_heads, dtype=np.int32).reshape(-1, 2))
            o.alignment_heads = iptr(self._ah)
            o.n_alignment_heads = int(self._ah.shape[0])
        o.median_filter_width = median_filter_width
        o.use_graph = int(use_graph)
        o.max_audio_samples = max_audio_samples
        # temperature > 0: best_of sampled rows per window (faster-whisper's sampling branch), beam_size unused
        o.temperature = float(temperature)
        o.best_of = int(best_of)
        o.sample_seed = int(sample_seed) & 0xFFFFFFFF
        self.opts = o
        self.max_batch = max_batch
        self.max_audio_samples = max_audio_samples
        h = C.c_void_p()
        check(lib.wmx_ctx_create(model.handle, C.byref(o), C.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def stream(self) -> int:
        return int(lib.wmx_ctx_stream(self._h) or 0)

    # ---- batching helpers ----
    def _pack(self, audios):
        B = len(audios)
        stride = max(1, max(len(a) for a in audios))
        pcm = np.zeros((B, stride), np.float32)
        for i, a in enumerate(audios):
            pcm[i, : len(a)] = a
        lens = np.array([len(a) for a in audios], np.int64)
        return pcm, stride, lens

    def logmel(self, audios, seek=None) -> np.ndarray:
        pcm, stride, lens = self._pack(audios)
        B = len(audios)
        out = np.empty((B, self.model.dims.n_mels, 3000), np.float32)
        sk = None if seek is None else np.ascontiguousarray(np.asarray(seek, np.int32))
        check(lib.wmx_logmel(self._h, fptr(pcm), stride, lptr(lens), iptr(sk) if sk is not None else None, B,
                             fptr(out)))
        return out

    def encode(self, mel: np.ndarray, want_output: bool = True):
        mel = np.ascontiguousarray(mel, np.float32)
        B = mel.shape[0]
        out = np.empty((B, 1500, self.model.dims.n_audio_state), np.float32) if want_output else None
        check(lib.wmx_encode(self._h, fptr(mel), B, fptr(out) if out is not None else None))
        return out

    def decoder_logits(self, tokens: np.ndarray) -> np.ndarray:
        tokens = np.ascontiguousarray(tokens, np.int32)
        B, T = tokens.shape
        lens = np.full(B, T, np.int32)
        out = np.empty((B, T, self.model.dims.n_vocab), np.float32)
        check(lib.wmx_decoder_logits(self._h, iptr(tokens), iptr(lens), B, T, fptr(out)))
        return out

    def forced_decode(self, prefix, tokens: np.ndarray, parents: np.ndarray | None = None, logits_every: int = 0):
        """Teacher-forced decode STEPS over the encoded windows (wmx_ctx_forced_decode): prefix = B token lists
        (left-padded to the longest, as transcribe pads prompts);
        tokens / parents [n_steps][R] with R = B x beam_size (parents None = every row extends itself).
        Returns (top1 [n_steps+1][R], logits [ceil((n_steps+1)/every)][R][V] or None)."""
        B, P = len(prefix), max(len(p) for p in prefix)
        plens = np.array([len(p) for p in prefix], np.int32)
        prefix = np.ascontiguousarray(np.array([list(p) + [0] * (P - len(p)) for p in prefix], np.int32))
        R = B * self.opts.beam_size
        tokens = np.ascontiguousarray(np.asarray(tokens, np.int32).reshape(-1, R))
        n = tokens.shape[0]
        if parents is None:
            parents = np.tile(np.arange(R, dtype=np.int32), (n, 1))
        parents = np.ascontiguousarray(np.asarray(parents, np.int32).reshape(n, R))
        top1 = np.empty((n + 1, R), np.int32)
        lg = None
        if logits_every > 0:
            lg = np.empty(((n + logits_every) // logits_every, R, self.model.dims.n_vocab), np.float32)
        check(lib.wmx_ctx_forced_decode(self._h, iptr(prefix), iptr(plens) if plens is not None else None, P, B, n, iptr(tokens), iptr(parents), iptr(top1),
                                        fptr(lg) if lg is not None else None, max(1, logits_every)))
        return top1, lg

    def set_sample_seed(self, seed: int):
        """Seed of the Gumbel draws of the following transcribe calls (wmx_ctx_set_sample_seed)."""
        self.opts.sample_seed = int(seed) & 0xFFFFFFFF
        check(lib.wmx_ctx_set_sample_seed(self._h, self.opts.sample_seed))

    def record(self, max_steps: int):
        """Parity recorder of the decode search (wmx_ctx_record); 0 turns it off."""
        check(lib.wmx_ctx_record(self._h, int(max_steps)))

    def recorded(self):
        """(logits [n][R][V], selections [n][R][2]) of the last transcribe (wmx_ctx_recorded)."""
        n, R = C.c_int(), C.c_int()
        check(lib.wmx_ctx_recorded(self._h, None, None, C.byref(n), C.byref(R)))
        lg = np.empty((n.value, R.value, self.model.dims.n_vocab), np.float32)
        sel = np.empty((n.value, R.value, 2), np.int32)
        check(lib.wmx_ctx_recorded(self._h, fptr(lg), iptr(sel), C.byref(n), C.byref(R)))
        return lg, sel

    def alignment_matrix(self, b: int) -> np.ndarray:
        """The word-alignment matrix window b's DTW ran on in the last transcribe (wmx_ctx_alignment_matrix):
        [n_text_tokens + 1][seek_frames // 2]."""
        n, nf = C.c_int(), C.c_int()
        check(lib.wmx_ctx_alignment_matrix(self._h, int(b), None, C.byref(n), C.byref(nf)))
        out = np.empty((n.value, nf.value), np.float32)
        check(lib.wmx_ctx_alignment_matrix(self._h, int(b), fptr(out), C.byref(n), C.byref(nf)))
        return out

    def _collect(self, res_ptr) -> list:
        r = res_ptr.contents
        out = []
        for i in range(r.n_windows):
            w = r.windows[i]
            toks = [w.tokens[j] for j in range(w.n_tokens)]
            jt = np.ctypeslib.as_array(w.jump_times, (w.n_text_tokens + 1,)).copy() if w.jump_times else None
            tp = (np.ctypeslib.as_array(w.text_token_probs, (w.n_text_tokens,)).copy()
                  if w.text_token_probs and w.n_text_tokens > 0 else None)
            out.append(WindowResult(toks, w.language, w.language_prob, w.sum_logprob, w.avg_logprob,
                                    w.no_speech_prob, w.seek_frames, jt, tp))
        lib.wmx_result_free(res_ptr)
        return out

    def _prompts(self, prompts, B):
        if not prompts or all(not p for p in prompts):
            return None, None
        ids = np.ascontiguousarray(np.concatenate([np.asarray(p or [], np.int32) for p in prompts]).astype(np.int32))
        plens = np.array([len(p or []) for p in prompts], np.int32)
        return ids, plens

    def transcribe(self, audios, prompts=None, seek=None) -> list:
        """Batched hot path over windows (list of f32 arrays, <= max_audio_samples each)."""
        B = len(audios)
        pcm, stride, lens = self._pack(audios)
        ids, plens = self._prompts(prompts, B)
        sk = None if seek is None else np.ascontiguousarray(np.asarray(seek, np.int32))
        res = C.POINTER(L.Result)()
        check(lib.wmx_transcribe(self._h, fptr(pcm), stride, lptr(lens), iptr(sk) if sk is not None else None, B,
                                 iptr(ids) if ids is not None else None, iptr(plens) if plens is not None else None,
                                 C.byref(res)))
        return self._collect(res)

    def transcribe_device(self, pcm_dev_ptr: int, stride: int, lens: np.ndarray, prompts=None) -> list:
        """Same with the pcm already resident in HBM (bench: inputs resident before the timed region)."""
        lens = np.ascontiguousarray(lens, np.int64)
        B = lens.shape[0]
        ids, plens = self._prompts(prompts, B)
        res = C.POINTER(L.Result)()
        check(lib.wmx_transcribe_device(self._h, C.c_void_p(pcm_dev_ptr), stride, lptr(lens), None, B,
                                        iptr(ids) if ids is not None else None,
                                        iptr(plens) if plens is not None else None, C.byref(res)))
        return self._collect(res)

    def stage_ms(self) -> list:
        out = np.zeros(7, np.float32)
        check(lib.wmx_ctx_stage_ms(self._h, fptr(out)))
        return out.tolist()

    def last_steps(self) -> int:
        return int(lib.wmx_ctx_last_steps(self._h))

    KERNELS = {"cross_attn": 0, "enc_fc1": 1, "enc_attn": 2, "logmel": 3, "dec_fc1": 4, "self_attn": 5, "encoder": 6,
               "dec_qkv": 7, "dec_proj": 8, "dec_fc2": 9, "reduce_ln": 10, "dec_fc1_lnf": 11}

    PROBE_LAUNCHES = ("dec_qkv", "dec_out", "dec_cross_q", "dec_cross_out", "dec_fc1", "dec_fc2", "cross_attn",
                      "self_attn", "reduce_ln_out", "reduce_ln_cross_out", "reduce_ln_fc2", "prev_layer_last")

    def set_probe(self, on: bool, layer: int = 1):
        """In-situ probes on every launch of decoder layer `layer` (>= 1) and the previous layer's last launch: every
        step of every following transcribe records each workgroup's first and last device-clock tick."""
        check(lib.wmx_ctx_set_probe(self._h, 0 if on else -1, layer))

    def probe_launches(self, e2e: bool = True) -> dict:
        """{launch: (average in-situ duration ms, samples, algorithmic bytes of one launch)} of the last transcribe:
        e2e = end of the launch minus end of its predecessor in the layer's chain (dispatch + execution, what
        rocprofv3 reports per kernel); else the first-workgroup-start .. last-workgroup-end span."""
        n_l = len(self.PROBE_LAUNCHES)
        ms = np.zeros(n_l, np.float32)
        by = np.zeros(n_l, np.float64)
        n = np.zeros(n_l, np.int32)
        ems = np.zeros(n_l, np.float32)
        en = np.zeros(n_l, np.int32)
        check(lib.wmx_ctx_probe_launches(self._h, fptr(ms), by.ctypes.data_as(C.POINTER(C.c_double)), iptr(n),
                                         fptr(ems), iptr(en)))
        if e2e:
            ms, n = ems, en
        return {k: (float(ms[i]), int(n[i]), float(by[i])) for i, k in enumerate(self.PROBE_LAUNCHES)}

    def set_lockstep(self, key: int, n_members: int):
        """Join (key != 0) or leave (key 0) a lockstep group of contexts that transcribe concurrently: their decode
        loops start together (wmx_ctx_set_lockstep)."""
        check(lib.wmx_ctx_set_lockstep(self._h, int(key), int(n_members)))

    @property
    def lockstep_timeouts(self) -> int:
        """Chunk barriers of this context that timed out since it was created (wmx_ctx_lockstep_timeouts)."""
        n = C.c_int64(0)
        check(lib.wmx_ctx_lockstep_timeouts(self._h, C.byref(n)))
        return int(n.value)

    def probe_ticks(self):
        """(ticks [steps][12][2] uint64 earliest start / latest end per probed launch, wall-clock kHz) of the last
        transcribe (wmx_ctx_probe_ticks; 0 = not recorded)."""
        n, khz = C.c_int(), C.c_double()
        check(lib.wmx_ctx_probe_ticks(self._h, None, C.byref(n), C.byref(khz)))
        t = np.zeros((max(n.value, 1), len(self.PROBE_LAUNCHES), 2), np.uint64)
        if n.value:
            check(lib.wmx_ctx_probe_ticks(self._h, t.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(n), C.byref(khz)))
        return t[:n.value], float(khz.value)

    def bench_kernel(self, kernel: str, batch: int, iters: int = 50):
        """Average launch duration (ms) of one hot-path kernel replayed on the context stream (HIP events),
        with its algorithmic bytes and flops per launch."""
        ms, by, fl = C.c_float(), C.c_double(), C.c_double()
        check(lib.wmx_ctx_bench_kernel(self._h, self.KERNELS[kernel], batch, iters, C.byref(ms), C.byref(by),
                                       C.byref(fl)))
        return float(ms.value), float(by.value), float(fl.value)

    def close(self):
        if getattr(self, "_h", None):
            lib.wmx_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
