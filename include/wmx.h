/*
 * wmx.h — C ABI of libwmx.so, the MI355X-native streaming-Whisper hot path.
 *
 * This is the drop-in boundary that replaces the faster-whisper 1.2.1 / CTranslate2 4.6.1 engine behind
 * the reference's ASR plugin surface.  The reference binds that engine from Python:
 *
 *   asr_components.py:247-264  load_model()  -> faster_whisper.WhisperModel(name, device, compute_type,
 *                                                download_root, num_workers, device_index)
 *   asr_components.py:267-289  transcribe()  -> model.transcribe(audio, language, initial_prompt,
 *                                                beam_size, temperature, word_timestamps=True,
 *                                                condition_on_previous_text=True, task=...)
 *
 * The Python adapter wmx.asr.MI355XWhisperASR keeps that exact Python surface and calls the entry points
 * below through ctypes.  Plain pointers and sizes only; no torch types.
 *
 * Conventions
 *   - every call returns wmx_status (0 = ok); on error wmx_last_error() returns a thread-local message.
 *   - input buffers are owned by the caller; wmx_result is owned by the library until wmx_result_free().
 *   - one wmx_ctx per host thread / stream group; a wmx_model is read-only after init and shareable.
 *   - "host" pointers are ordinary CPU memory; "_device" entry points take device pointers on the
 *     context's device and do not synchronise.
 */
#ifndef WMX_H
#define WMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int wmx_status;
enum {
  WMX_OK = 0,
  WMX_ERR_ARG = 1,      /* bad argument / shape */
  WMX_ERR_HIP = 2,      /* HIP runtime error */
  WMX_ERR_STATE = 3,    /* call in the wrong state (e.g. decode before encode) */
  WMX_ERR_NOMEM = 4,
  WMX_ERR_NUMERIC = 5,  /* the decode produced non-finite logits (wmx_last_error names the step and row) */
};

/* WMX_DTYPE_MX8 (BASELINE config 5, "large-v3 fp8"): bf16 storage and activations, with
 *  - the encoder projections (q/k/v, out, fc1, fc2) on the CDNA4 MX-fp8 MFMA (OCP e4m3 elements, e8m0 scale per
 *    32 K) with MX-fp8 activations;
 *  - the fp8 decode: every decoder projection and the logits projection on 8-bit weights (e4m3, one power-of-two
 *    scale per weight row, widened to bf16 in registers) and the cross-attention K / V images in e4m3 (one
 *    power-of-two scale per (layer, window, head) image).  WMX_DEC_FP8=0 in the environment keeps the decode bf16.
 * The reference's own 8-bit GPU mode is CTranslate2's int8_float16 (int8 weights with per-row scales): the host
 * layer maps compute_type "int8_float16" / "int8" to this dtype (wmx/engine.py). */
/* WMX_DTYPE_I8 / WMX_DTYPE_I8_BF16 (the reference's CTranslate2 int8 modes, int8_float16 / int8:
 * 一键实时识别麦克风.py:304, asr_components.py:256-261): every decoder projection and the logits projection on
 * int8 weights with CTranslate2's per-row scales (q = rint(w * scale), scale = 127 / max|row| or a CT2 int8
 * checkpoint's own weight_scale, wmx_model_set_row_scales), widened exactly to 16 bits in registers, the row's
 * 1 / scale applied to the fp32 result; f16 (I8) or bf16 (I8_BF16) activations and storage; the encoder, the
 * cross-K/V projection and the embedding lookup on the 16-bit weights (q / scale rounded to 16 bits). */
enum { WMX_DTYPE_BF16 = 0, WMX_DTYPE_F16 = 1, WMX_DTYPE_MX8 = 2, WMX_DTYPE_I8 = 3, WMX_DTYPE_I8_BF16 = 4 };
enum { WMX_TASK_TRANSCRIBE = 0, WMX_TASK_TRANSLATE = 1 };

typedef struct wmx_model wmx_model;
typedef struct wmx_ctx wmx_ctx;

/* openai-whisper ModelDimensions (what a CT2 / HF checkpoint's config.json carries). */
typedef struct {
  int32_t n_mels;
  int32_t n_vocab;
  int32_t n_audio_ctx;   /* 1500 */
  int32_t n_audio_state;
  int32_t n_audio_head;
  int32_t n_audio_layer;
  int32_t n_text_ctx;    /* 448 */
  int32_t n_text_state;
  int32_t n_text_head;
  int32_t n_text_layer;
} wmx_dims;

/* decoding options — faster-whisper TranscriptionOptions fields that reach CT2 generate()
 * (asr_components.py:279-288 passes beam_size, temperature=0.0, task, word_timestamps). */
typedef struct {
  int32_t max_batch;                 /* windows per call (streams sharing one launch) */
  int32_t beam_size;                 /* 1 = greedy (temperature 0), else beam search */
  float patience;                    /* faster-whisper default 1.0 */
  float length_penalty;              /* 1.0 -> score / len (CT2 default used by faster-whisper) */
  int32_t max_new_tokens;            /* <= n_text_ctx - prompt; faster-whisper: 448 - prompt */
  int32_t task;                      /* WMX_TASK_* */
  int32_t language;                  /* language token id, or -1 = detect per window */
  int32_t without_timestamps;        /* 0 (faster-whisper default) */
  int32_t max_initial_timestamp_index; /* 50 = 1.0 s; -1 = none */
  int32_t suppress_blank;            /* 1 */
  const int32_t* suppress_tokens;    /* ids to suppress every step (faster-whisper suppress_tokens=[-1] expanded) */
  int32_t n_suppress_tokens;
  int32_t word_timestamps;           /* run the alignment forward + DTW */
  const int32_t* alignment_heads;    /* [n][2] (layer, head); NULL = every head of the second half */
  int32_t n_alignment_heads;
  int32_t median_filter_width;       /* 7 */
  int32_t use_graph;                 /* capture the decode step in a hipGraph */
  int32_t max_audio_samples;         /* longest pcm per window accepted (default 480000) */
  /* temperature > 0: faster-whisper's sampling branch (generate_with_fallback: beam_size 1, num_hypotheses = best_of,
   * sampling_topk 0, sampling_temperature = temperature): best_of independent rows per window, each drawing its next
   * token from softmax(rule-masked logits / temperature) by Gumbel-max on a counter-based hash of (sample_seed, row,
   * slot, token); the window keeps the row with the best sum_logprob / length.  beam_size is ignored then. */
  float temperature;                 /* 0 = deterministic search (default) */
  int32_t best_of;                   /* rows per window when sampling, 1..8 (faster-whisper default 5) */
  uint32_t sample_seed;
} wmx_opts;

/* per-window result of wmx_transcribe */
typedef struct {
  int32_t language;                  /* language token used (detected or given) */
  float language_prob;               /* probability of that language (1.0 if given) */
  int32_t n_tokens;                  /* sampled tokens, EOT excluded (text + timestamp tokens) */
  const int32_t* tokens;
  float sum_logprob;
  float avg_logprob;                 /* sum_logprob / (n_tokens + 1) (faster-whisper) */
  float no_speech_prob;
  int32_t seek_frames;               /* content frames of this window (segment_size) */
  /* word_timestamps: one entry per TEXT token (tokens < eot, in order) + 1 for the trailing eot */
  int32_t n_text_tokens;
  const float* jump_times;           /* [n_text_tokens + 1] seconds, faster-whisper find_alignment jump_times */
  const float* text_token_probs;     /* [n_text_tokens] */
} wmx_window_result;

typedef struct {
  int32_t n_windows;
  const wmx_window_result* windows;
} wmx_result;

const char* wmx_last_error(void);
const char* wmx_version(void);
int wmx_device_count(void);

/* ---- model ---- */
wmx_status wmx_model_create(const wmx_dims* dims, int device, int dtype, wmx_model** out);
void wmx_model_free(wmx_model* m);
/* build-owned deterministic synthetic weights (oracle/whisper_np.py make_weights, same PRNG) */
wmx_status wmx_model_init_synthetic(wmx_model* m, uint64_t seed);
/* load one tensor by its HF/openai state-dict name from host fp32 (logical HF layout) */
wmx_status wmx_model_set_tensor(wmx_model* m, const char* name, const float* data, int64_t n);
/* read back one tensor (logical HF layout, values as stored) — tests / checkpoint export */
wmx_status wmx_model_get_tensor(wmx_model* m, const char* name, float* out, int64_t n);
int64_t wmx_model_n_params(const wmx_model* m);
/* int8 models only: set the CTranslate2 row scales of a decoder projection or of decoder.embed_tokens.weight (HF
 * names, e.g. "decoder.layers.3.fc1.weight"; n = its rows), after its weight; wmx_model_get_int8 reads back the
 * device's int8 bytes [rows][cols] and scales of one such weight (tests). */
wmx_status wmx_model_set_row_scales(wmx_model* m, const char* name, const float* scale, int64_t n);
wmx_status wmx_model_get_int8(wmx_model* m, const char* name, int8_t* q, float* scale, int64_t rows, int64_t cols);
/* the parameter region of the weight arena: [device_ptr, device_ptr + bytes) holds every parameter (what an RCCL
 * broadcast of the weights must carry); the derived copies (row-major, MX-fp8, 8-bit, LayerNorm-folded, log-mel
 * constants) live after it and are rebuilt on each rank by wmx_model_arena_loaded */
wmx_status wmx_model_arena(wmx_model* m, void** device_ptr, size_t* bytes);
/* after the parameter region was overwritten externally (e.g. ncclBroadcast): derive the copies, mark initialised */
wmx_status wmx_model_arena_loaded(wmx_model* m);

/* ---- context ---- */
void wmx_opts_default(wmx_opts* o);
wmx_status wmx_ctx_create(wmx_model* m, const wmx_opts* o, wmx_ctx** out);
void wmx_ctx_destroy(wmx_ctx* c);
/* the HIP stream the context launches on (hipStream_t as void*) */
void* wmx_ctx_stream(wmx_ctx* c);

/* log-mel of B windows (faster-whisper FeatureExtractor, padding=160, pad_or_trim to 3000 frames).
 * pcm: B rows of `stride` floats, row b holds lens[b] samples; seek: first frame per window (NULL = 0).
 * mel_out: host [B][n_mels][3000]. */
wmx_status wmx_logmel(wmx_ctx* c, const float* pcm, int64_t stride, const int64_t* lens, const int32_t* seek,
                      int B, float* mel_out);
wmx_status wmx_logmel_device(wmx_ctx* c, const float* pcm_dev, int64_t stride, const int64_t* lens,
                             const int32_t* seek, int B, float* mel_out_dev);

/* encoder on B normalised mel windows (host [B][n_mels][3000]); keeps encoder output + cross K/V in the
 * context.  enc_out (nullable): host [B][1500][n_audio_state] f32 copy of the (rounded) encoder output. */
wmx_status wmx_encode(wmx_ctx* c, const float* mel, int B, float* enc_out);
wmx_status wmx_encode_device(wmx_ctx* c, const float* mel_dev, int B);

/* teacher-forced decoder forward over the encoded windows: tokens [B][T] (pad with any id beyond
 * lens[b]); logits_out host [B][T][n_vocab] f32 (rows beyond lens[b] undefined). */
wmx_status wmx_decoder_logits(wmx_ctx* c, const int32_t* tokens, const int32_t* lens, int B, int T,
                              float* logits_out);

/* parity hook for the decode-STEP kernels (the launches a transcribe step replays: packed split-K GEMMs,
 * ancestry-gathered self attention, cross attention, reduce + LayerNorm, logits), teacher-forced: the B encoded
 * windows' rows (R = B x beam_size, row r belongs to window r / beam_size) are prefilled with prefix [B][P]
 * (window b's first prefix_lens[b] ids, left-padded to P as transcribe pads prompts; prefix_lens NULL = all P), then
 * n_steps steps each append tokens[i][r] to the history of row parents[i][r] (a row of the same window; the
 * beam reorder of a real step, ancestry rows only) and run one decode step.  Step 0 is the prefill's last position
 * (shared by a window's rows).  top1 [(n_steps+1)][R] = argmax of the raw logits (lowest id on ties); logits
 * (nullable) [(n_steps+1)/every rounded up][R][n_vocab] = the raw logits of steps 0, every, 2*every, ...
 * Replaces nothing in the reference; tests only. */
wmx_status wmx_ctx_forced_decode(wmx_ctx* c, const int32_t* prefix, const int32_t* prefix_lens, int P, int B,
                                 int n_steps,
                                 const int32_t* tokens, const int32_t* parents, int32_t* top1, float* logits,
                                 int every);

/* the hot path: pcm -> log-mel -> encoder -> [language detect] -> prompt prefill -> greedy/beam decode
 * (hipGraph) -> [alignment forward + DTW].  prompt_ids: concatenated previous-text token ids per window
 * (prompt_lens[b] each; faster-whisper keeps the last 223); NULL = no prompt. */
wmx_status wmx_transcribe(wmx_ctx* c, const float* pcm, int64_t stride, const int64_t* lens, const int32_t* seek,
                          int B, const int32_t* prompt_ids, const int32_t* prompt_lens, wmx_result** out);
/* same with the pcm already resident in device memory (bench: inputs in HBM before the timed region) */
wmx_status wmx_transcribe_device(wmx_ctx* c, const float* pcm_dev, int64_t stride, const int64_t* lens,
                                 const int32_t* seek, int B, const int32_t* prompt_ids,
                                 const int32_t* prompt_lens, wmx_result** out);
void wmx_result_free(wmx_result* r);

/* profiling hooks: per-stage device time of the last wmx_transcribe (ms), HIP events on the ctx stream.
 * stages: 0 logmel, 1 encoder, 2 cross-kv, 3 lang-detect, 4 prefill, 5 decode loop, 6 alignment. */
wmx_status wmx_ctx_stage_ms(wmx_ctx* c, float* out7);
/* total decode steps executed by the last wmx_transcribe */
int wmx_ctx_last_steps(wmx_ctx* c);

/* roofline hook: replay ONE kernel of the hot path `iters` times on the context stream (geometry and data of
 * the last wmx_transcribe, B windows) between two HIP events; returns the average launch duration and the
 * ALGORITHMIC bytes / flops of one launch.  kernel: 0 decoder cross-attention (one layer, decode step),
 * 1 encoder fc1 GEMM, 2 encoder self-attention (one layer), 3 log-mel (raw pass), 4 decoder fc1 GEMM (step),
 * 5 decoder self-attention (one layer, at the last decoded length), 6 the whole encoder over B windows,
 * 7 / 8 / 9 decoder qkv / d x d / fc2 projection (split-K partial launch of a step), 10 reduce_ln of a d x d
 * projection's partials (residual add + LayerNorm). */
wmx_status wmx_ctx_bench_kernel(wmx_ctx* c, int kernel, int B, int iters, float* avg_ms, double* bytes,
                                double* flops);

/* parity recorder of the decode SEARCH (tests only): with max_steps > 0 every following wmx_transcribe copies,
 * per decode step i < max_steps (step 0 = the selection from the prompt prefill), the raw logits of each of its
 * R = B x beam_size rows before the rules and selection, and the selection: greedy (row, token) of live rows, beam
 * (parent row, token) of the rows of windows still searching, (-1, -1) otherwise.  max_steps = 0 turns it off.
 * wmx_ctx_recorded: n_steps = min(steps of the last transcribe, max_steps), rows = its R; logits (nullable)
 * [n_steps][R][n_vocab], sel (nullable) [n_steps][R][2]. */
wmx_status wmx_ctx_record(wmx_ctx* c, int max_steps);
wmx_status wmx_ctx_recorded(wmx_ctx* c, float* logits, int32_t* sel, int* n_steps, int* rows);

/* the sampling seed of the following wmx_transcribe calls (temperature > 0; initially wmx_opts.sample_seed).  The
 * Gumbel noise is a pure function of (seed, row, slot, token), so a caller that wants fresh draws per window and per
 * temperature of a fallback schedule (as faster-whisper / CT2 draw new randomness per generate call) passes a
 * different seed per call; the same seed replays the same draws. */
wmx_status wmx_ctx_set_sample_seed(wmx_ctx* c, uint32_t seed);

/* word-alignment matrix of window b of the last wmx_transcribe (tests only): the matrix the DTW ran on -- for the
 * rows <|notimestamps|> + text tokens (n = n_text_tokens + 1) and the first nf = seek_frames / 2 encoder frames, the
 * mean over the alignment heads of softmax(cross-attention scores over nf frames), normalised per frame over the
 * token axis and median-filtered along frames (openai timing.find_alignment `matrix`, via faster-whisper).
 * out [n][nf] (nullable: sizes only). */
wmx_status wmx_ctx_alignment_matrix(wmx_ctx* c, int b, float* out, int* n, int* nf);

/* host-only check of the decode GEMM's addressing (no GPU needed; tests only): for a packed-weight launch of
 * M rows x N columns x K (lda = A's row stride), split = 0 as the epilogue launches (S = 1) or 1 as the split-K
 * partial launches with a part_cap-element partial buffer, out9 = {S, MT, NCT, NW, KU, weight elements touched
 * (end offset), A elements touched (end offset), partial elements written (end offset), k-steps loaded outside the
 * wave's slice}, computed by walking the launch through the kernel's own index helpers (wmx_kernels.h). */
wmx_status wmx_debug_packed_launch(int M, int N, int K, int64_t part_cap, int split, int64_t lda, int64_t* out9);
/* Host-only (no GPU call): the word-alignment DTW of wmx_transcribe on a caller alignment matrix x[N][ld] (first M
 * columns; the DTW cost is -x, as openai timing calls dtw(-matrix)), returning the backtraced path (ti[k], tj[k]),
 * k < *len <= N + M, in path order from (0, 0).
 * Replaces the reference's openai `timing.dtw_cpu` + `backtrace` (via faster-whisper's find_alignment). */
wmx_status wmx_debug_dtw(const float* x, int N, int M, int ld, int32_t* ti, int32_t* tj, int* len);

/* ---- pre-ASR DSP of the microphone loop, batched over B streams ----
 * band-pass "vocal separation" (reference vocal_separation.py:335-358, SimpleFilterSeparator.separate):
 * y = scipy.signal.filtfilt(b, a, x) with the caller's normalised coefficients (a[0] = 1, ntaps = len(b) = len(a)
 * <= 17, zi = scipy.signal.lfilter_zi(b, a), ntaps - 1 values; padlen = 3 * ntaps).  Stream i has lens[i] samples
 * at x + i * stride; y has the same layout.  fp64 recursion, as scipy. */
wmx_status wmx_filtfilt(wmx_ctx* c, const float* x, int64_t stride, const int64_t* lens, int B, const double* b,
                        const double* a, const double* zi, int ntaps, float* y);
wmx_status wmx_filtfilt_device(wmx_ctx* c, const float* x_dev, int64_t stride, const int64_t* lens, int B,
                               const double* b, const double* a, const double* zi, int ntaps, float* y_dev);
/* audio-dedup features (reference audio_deduplicator.py:60-160, AudioDeduplicator._extract_features):
 * out[i][0..4] = (rms, spectral centroid, zero-crossing rate, 85 % roll-off, bandwidth) / max|.| of stream i,
 * lens[i] <= 8000 samples at sample rate sr.  The history / similarity decision stays on the host. */
wmx_status wmx_dedup_features(wmx_ctx* c, const float* x, int64_t stride, const int64_t* lens, int B, float sr,
                              float* out);

/* ---- Silero VAD v5 (16 kHz) on device, batched over streams ----
 * Replaces the torch.hub Silero model of asr_components.py:96 as called by whisper_streaming's VADIterator
 * (`model(x, 16000).item()` per 512 samples, `model.reset_states()`).  A wmx_vad holds the f32 weights and, per
 * slot (one stream each, up to max_streams), the LSTM state (h, c) and the last 64 input samples.
 * wmx_vad_set_tensor takes the v5 state-dict names without the `_model.` prefix ("stft.forward_basis_buffer",
 * "encoder.{0..3}.reparam_conv.{weight,bias}", "decoder.rnn.{weight_ih,weight_hh,bias_ih,bias_hh}",
 * "decoder.decoder.2.{weight,bias}"), row-major as torch stores them; every tensor must be set before processing.
 * wmx_vad_process: stream i of S (slot slots[i], distinct) brings nwin * 512 new samples at pcm + i * stride
 * (host memory); probs[i * nwin + j] = speech probability of its window j, windows run in order (the model's
 * state and context carry across windows and calls). */
typedef struct wmx_vad wmx_vad;
wmx_status wmx_vad_create(int device, int max_streams, int max_windows, wmx_vad** out);
void wmx_vad_free(wmx_vad* v);
wmx_status wmx_vad_set_tensor(wmx_vad* v, const char* name, const float* data, int64_t n);
/* zero the state and context of one slot (slot < 0: all slots) */
wmx_status wmx_vad_reset(wmx_vad* v, int slot);
wmx_status wmx_vad_process(wmx_vad* v, const float* pcm, int64_t stride, const int32_t* slots, int S, int nwin,
                           float* probs);
/* the same on device buffers (pcm_dev, probs_dev on the VAD's device; slots in host memory), no synchronisation;
 * the stream it runs on is wmx_vad_stream(v) */
wmx_status wmx_vad_process_device(wmx_vad* v, const float* pcm_dev, int64_t stride, const int32_t* slots, int S,
                                  int nwin, float* probs_dev);
void* wmx_vad_stream(wmx_vad* v);

/* in-situ roofline probes: with kernel = 0, every launch of decoder layer `layer` (>= 1) of every decode step of the
 * timed wmx_transcribe -- the six packed projection GEMMs (ids 0 qkv, 1 out, 2 cross-q, 3 cross-out, 4 fc1, 5 fc2),
 * the cross attention (6), the self attention (7), the three reduce + LayerNorm launches (8, 9, 10) and the
 * previous layer's last launch (11) -- store each workgroup's first and last device wall-clock tick
 * (hipDeviceAttributeWallClockRate), one plain store per workgroup; kernel < 0 disables them.
 * wmx_ctx_probe_stats: the cross attention's average span (ms), steps sampled, ALGORITHMIC bytes of one launch.
 * wmx_ctx_probe_launches, arrays of 12: span_ms / span_n = average first-workgroup-start .. last-workgroup-end;
 * e2e_ms / e2e_n (nullable) = average last-workgroup-end minus that of the launch before it in the layer's chain
 * (dispatch + execution: the per-kernel span rocprofv3 reports, plus the inter-kernel gap); bytes = ALGORITHMIC
 * bytes of one launch (ids 0-6; 0 for the others). */
wmx_status wmx_ctx_set_probe(wmx_ctx* c, int kernel, int layer);
/* context groups decoding concurrently on one GPU run the same launch sequence; an idle offset of `us`
 * microseconds before this context's decode loop shifts its phase against the other group's, so their HBM-heavy
 * (cross attention) and latency-bound launches overlap each other instead of coinciding.  0 = none. */
wmx_status wmx_ctx_set_phase_offset(wmx_ctx* c, double us);
/* context groups decoding concurrently on one GPU (e.g. the bench's two groups, one host thread each): contexts set to
 * the same key (!= 0) with n_members >= 2 meet at a host barrier right before their decode loops (5 ms timeout), so
 * their step graphs start together and stay in step -- each layer's weights are then read once for all groups (the
 * later reader hits the caches) -- and again before every later 8-step chunk, waiting only for the members still
 * decoding (WMX_LOCKSTEP_CHUNKS=0: the start barrier only). Every member must call wmx_transcribe concurrently with
 * the others; a member that does not costs the others the timeout once. key 0 leaves the group. */
wmx_status wmx_ctx_set_lockstep(wmx_ctx* c, int key, int n_members);
/* chunk barriers of this context that timed out since it was created (the member then leaves the barrier for the
 * rest of its call): 0 while the group's members arrive together and leave when their decode loops end */
wmx_status wmx_ctx_lockstep_timeouts(wmx_ctx* c, int64_t* n);
/* the lockstep barriers alone (host tests, no GPU), group `key` of n members: op 0 = the start barrier (all n),
 * 1 = a chunk barrier (the members still decoding), 2 = leave (this member's decode loop ended); *ok = 1 when every
 * expected member arrived within timeout_us, else 0 (the member leaves that round; the next one starts clean) */
wmx_status wmx_debug_lockstep_arrive(int key, int n_members, int op, int timeout_us, int* ok);
wmx_status wmx_ctx_probe_stats(wmx_ctx* c, float* avg_ms, int* n, double* bytes);
wmx_status wmx_ctx_probe_launches(wmx_ctx* c, float* span_ms, double* bytes, int* span_n, float* e2e_ms, int* e2e_n);
/* the probes' raw device wall-clock ticks of the last transcribe (diagnostics: the relative phase of two context
 * groups, per-step durations): lo_hi[(s * 12 + k) * 2 + {0, 1}] = earliest workgroup start / latest workgroup end of
 * launch id k at the s-th probed decode step, 0 when not recorded; *n_steps = steps written (lo_hi may be null to
 * query; capacity 448 steps), *wall_khz = the tick rate. */
wmx_status wmx_ctx_probe_ticks(wmx_ctx* c, uint64_t* lo_hi, int* n_steps, double* wall_khz);
/* diagnostics (WMX_PHASE_PROBE=1 in the environment at wmx_ctx_set_probe): the probed layer's decode cross attention
 * phase stamps of the last transcribe, out[(s * n_wg + wg) * n_words + i] for decode step s (at most cap_steps),
 * workgroup wg (linear id), word i = 0..7 device wall-clock ticks at the kernel's phase boundaries (wave 0: start,
 * query projection done, query tile ready, first scores, P.V done, waves combined, ticket taken, end), 8 = XCC_ID,
 * 9 = HW_ID; zero words for workgroups past the grid.  out may be null to query the sizes. */
wmx_status wmx_ctx_probe_phases(wmx_ctx* c, uint64_t* out, int cap_steps, int* n_steps, int* n_wg, int* n_words,
                                double* wall_khz);

#ifdef __cplusplus
}
#endif
#endif /* WMX_H */
