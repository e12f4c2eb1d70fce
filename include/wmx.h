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
 *
 * This header is the product surface.  Test, parity and measurement hooks (teacher-forced decode
 * steps, the search recorder, the alignment matrix, per-stage times, kernel replays, in-situ probes, host-only
 * checks) are declared in wmx_diag.h; they replace nothing in the reference.
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

/* the sampling seed of the following wmx_transcribe calls (temperature > 0; initially wmx_opts.sample_seed).  The
 * Gumbel noise is a pure function of (seed, row, slot, token), so a caller that wants fresh draws per window and per
 * temperature of a fallback schedule (as faster-whisper / CT2 draw new randomness per generate call) passes a
 * different seed per call; the same seed replays the same draws. */
wmx_status wmx_ctx_set_sample_seed(wmx_ctx* c, uint32_t seed);

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

/* ---- context groups decoding concurrently on one GPU ----
 * (e.g. the bench's two groups, one host thread each): contexts set to
 * the same key (!= 0) with n_members >= 2 meet at a host barrier right before their decode loops (5 ms timeout), so
 * their step graphs start together and stay in step -- each layer's weights are then read once for all groups (the
 * later reader hits the caches) -- and again before every later 8-step chunk, waiting only for the members still
 * decoding (WMX_LOCKSTEP_CHUNKS=0: the start barrier only). Every member must call wmx_transcribe concurrently with
 * the others; a member that does not costs the others the timeout once. key 0 leaves the group. */
wmx_status wmx_ctx_set_lockstep(wmx_ctx* c, int key, int n_members);
/* chunk barriers of this context that timed out since it was created (the member then leaves the barrier for the
 * rest of its call): 0 while the group's members arrive together and leave when their decode loops end */
wmx_status wmx_ctx_lockstep_timeouts(wmx_ctx* c, int64_t* n);

#ifdef __cplusplus
}
#endif
#endif /* WMX_H */
