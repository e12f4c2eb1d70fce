// Host-side interface of the decode-loop kernels (wmx_decode.hip).
#pragma once
#include "wmx_common.h"

namespace wmx {

struct RuleOpts {
  int V, eot, tb, no_ts, blank;
  int suppress_blank;
  int max_init;          // -1 = none
  int without_ts;
  const uint32_t* mask;  // suppress-token bitmask [ceil(V/32)]
  // sampling (temperature > 0): selection key = logit / T + Gumbel(hash(*seed, row, *slot, token)); inv_temp 0 = off.
  // The seed is read from device memory so that the captured decode graph draws with the seed of each call
  // (wmx_ctx_set_sample_seed), not the one baked in at capture.
  float inv_temp = 0.f;
  const uint32_t* seed = nullptr;
  const int* slot = nullptr;
  // non-finite guard: a row whose normaliser is not finite or that has no candidate (NaN / -inf logits) records
  // 1 + row + 1024 * slot in *err (the first one wins, compare-and-swap from 0); the host turns it into
  // WMX_ERR_NUMERIC.  The row's token still becomes EOT, so no id outside the vocabulary reaches the embedding
  int* err = nullptr;
  const int* err_slot = nullptr;
};

struct RowPtrs {  // per-row decode state (device arrays of R)
  int* ns;
  int* last;
  int* pen;
  int* last_ts;
  int* done;
  float* sum_lp;
};

struct BeamState {  // device arrays
  int* win_done;     // [nwin]
  int* win_active;   // [nwin]
  int* fin_count;    // [nwin]
  float* fin_score;  // [nwin*max_cand]
  int* fin_parent;
  int* fin_len;
  int* fin_hist;     // [nwin*max_cand][ld]
  int* new_parent;   // [R]
  int* new_tok;
  float* new_score;
};

// rules + log-softmax + top-KP per row, two phases over kSlices vocab slices; ws: logits_select_ws_floats(R, KP)
size_t logits_select_ws_floats(int R, int KP);
void launch_logits_select(const float* logits, int ldl, const RuleOpts& o, const RowPtrs& rp, int R, int KP, int* tok,
                          float* lp, const int* row_map, float* ws, hipStream_t st);
void launch_greedy_update(const RowPtrs& rp, const int* tok, const float* lp, int R, int tb, int eot, int* hist,
                          int hist_ld, int* slot, int* n_done, hipStream_t st);
void launch_beam_step(const RowPtrs& rp, const RowPtrs& tmp, const int* ctok, const float* clp, int nwin, int K,
                      int max_cand, int tb, int eot, int* slot, int* hist, int* hist_tmp, int* anc, int* anc_tmp, int ld,
                      const BeamState& bs, int* n_done, hipStream_t st);
void launch_lang_detect(const float* logits, int ldl, int lang0, int nlang, int nwin, int K, int* hist, int hist_ld,
                        const int* lang_slot, int* lang_out, float* prob_out, hipStream_t st,
                        int* err = nullptr);
void launch_token_prob(const float* logits, int ldl, int V, int token, int rows, float* out, hipStream_t st);
void launch_text_prob(const float* logits, int ldl, int eot, const int* target, int rows, float* out, hipStream_t st);
// parity instrumentation (wmx_ctx_record)
void launch_record_logits(const float* logits, int ldl, int V, int R, const int* row_map, const int* slot,
                          const int* base, int cap, float* out, hipStream_t st);
void launch_record_select(int R, int K, const int* ctok, const RowPtrs& rp, const BeamState& bs, const int* slot,
                          const int* base, int after, int cap, int* out, hipStream_t st);
// alignment matrix [nwin][Tn][Tk]: zero, accumulate heads (softmax over nframes/2, normalise over tokens, median
// filter), scale by 1/n_heads
void launch_align_matrix_zero(float* out, int nwin, int Tn, int Tk, hipStream_t st);
// (scores [nh][rows_total][Tk] are normalised in place)
void launch_align_matrix_acc(float* scores, int nh, int rows_total, int Tk, int Tn, const int* ntok,
                             const int* nframes, int width, int nwin, hipStream_t st, float* out);
void launch_align_matrix_scale(float* out, int nwin, int Tn, int Tk, const int* ntok, const int* nframes, float scale,
                               hipStream_t st);

}  // namespace wmx
