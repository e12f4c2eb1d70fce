/*
 * wmx_diag.h -- test, parity and measurement hooks of libwmx.so (not part of the drop-in surface, include/wmx.h).
 *
 * These entry points replace nothing in the reference.  The GPU parity tests (tests/test_gpu_*.py), bench.py's
 * roofline and stage lines and the host-only CPU tests call them through ctypes (wmx/_lib.py); a product caller
 * needs none of them.  They take the same handles and follow the same conventions as wmx.h (wmx_status return,
 * wmx_last_error() on failure).
 */
#ifndef WMX_DIAG_H
#define WMX_DIAG_H

#include "wmx.h"

#ifdef __cplusplus
extern "C" {
#endif

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
 * projection's partials (residual add + LayerNorm), 11 decoder fc1 of the mixed step (LayerNorm folded). */
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
/* Debug: with WMX_GUARD=1 in the environment when the model / context was created, every arena buffer is followed by a
 * 64 KiB guard gap holding a byte pattern; *model_buf / *ctx_buf = the index (allocation order) of the first buffer
 * whose gap was overwritten, -1 when every gap is intact (either handle may be NULL). */
wmx_status wmx_debug_guard_check(wmx_model* m, wmx_ctx* c, int* model_buf, int* ctx_buf);
/* Shader clock beside a workload (bench.py's encoder field): start launches n single-wave workgroups on a stream of
 * their own (workgroup i on XCD i mod 8) that sleep for ms milliseconds of the 100 MHz constant clock and returns at
 * once; result waits for them and writes each one's shader clock, d(s_memtime) / d(s_memrealtime) x 100 MHz, to
 * mhz[n].  One probe pending at a time. */
wmx_status wmx_debug_clock_start(int device, double ms, int n);
wmx_status wmx_debug_clock_result(float* mhz, int n);
/* Host-only (no GPU call): the word-alignment DTW of wmx_transcribe on a caller alignment matrix x[N][ld] (first M
 * columns; the DTW cost is -x, as openai timing calls dtw(-matrix)), returning the backtraced path (ti[k], tj[k]),
 * k < *len <= N + M, in path order from (0, 0).
 * Replaces the reference's openai `timing.dtw_cpu` + `backtrace` (via faster-whisper's find_alignment). */
wmx_status wmx_debug_dtw(const float* x, int N, int M, int ld, int32_t* ti, int32_t* tj, int* len);

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

#ifdef __cplusplus
}
#endif
#endif /* WMX_DIAG_H */
