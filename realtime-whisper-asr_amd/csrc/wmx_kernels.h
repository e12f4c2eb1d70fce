// Host-side launch interface of the libwmx HIP kernels.
#pragma once
#include "wmx_common.h"

namespace wmx {

enum EpiKind {
  EPI_STORE16 = 0,     // out16 = acc + bias
  EPI_GELU16 = 1,      // out16 = gelu(acc + bias)
  EPI_RESID32 = 2,     // out32 += acc + bias          (fp32 residual stream)
  EPI_GELU_POS32 = 3,  // out32 = gelu(acc + bias) + pos[m % posT]   (encoder conv2)
  EPI_STORE32 = 4,     // out32 = acc (+ bias)          (logits)
  EPI_QKV_CACHE = 5,   // decoder self-attn: q -> out16, k/v -> KV cache at slot *slot0 + (m % Tn)
};

struct Epi {
  int kind = EPI_STORE16;
  const float* bias = nullptr;
  void* out = nullptr;
  long ldc = 0;
  const float* pos = nullptr;
  int posT = 1;
  // EPI_QKV_CACHE
  int d = 0, Tn = 1, R = 1, rmul = 1;  // cache row = (m / Tn) * rmul
  const int* slot0 = nullptr;
  uint16_t* kc = nullptr;
  uint16_t* vc = nullptr;
};

enum GemmTile { TILE_128x128 = 0, TILE_64x64 = 1, TILE_32x64 = 2, TILE_SKINNY = 3 };

struct GemmCall {
  const uint16_t* A;
  long lda;
  const uint16_t* W;
  long ldw;
  int M, N, K;
  Epi epi;
  int tile = TILE_128x128;
  int splits = 1;
  float* ws = nullptr;  // split-K workspace
  long ws_elems = 0;
};

void launch_gemm(DT dt, const GemmCall& g, hipStream_t st);
void gemm_init_attributes();

// log-mel
size_t logmel_smem_bytes();
void launch_logmel(const float* pcm, long stride, const long* lens_dev, const int* seek_dev, int B, int max_frames,
                   const float* basis, const int* mfirst, const int* mcount, const int* moff, const float* mw,
                   int n_mels, float* raw, int fcap, int* wmax, float* out, hipStream_t st);

// elementwise / norm / layout
void launch_layernorm(DT dt, const float* x, const float* g, const float* b, uint16_t* out, int rows, int d,
                      hipStream_t st);
void launch_layernorm_rows(DT dt, const float* x, const int* row_idx, const float* g, const float* b, uint16_t* out,
                           int rows, int d, hipStream_t st);
void launch_im2col_conv1(DT dt, const float* mel, int B, int n_mels, int Kp, uint16_t* out, hipStream_t st);
void launch_im2col_conv2(DT dt, const uint16_t* h1, int B, int d, uint16_t* out, hipStream_t st);
void launch_cvt16_to_f32(DT dt, const uint16_t* in, float* out, long n, hipStream_t st);
// x[r*Tn+i] = tok_emb[hist[r*hist_ld + slot]] + pos_emb[slot - pad[r]],  slot = *slot0 + i
void launch_embed(DT dt, const uint16_t* tok_emb, const uint16_t* pos_emb, const int* hist, long hist_ld, int R, int Tn,
                  const int* pad, const int* slot0, int d, float* x, hipStream_t st);

// attention
struct AttnArgs {
  const uint16_t* q;   // [*, q_ld] rows
  long q_ld;
  long q_bstride;      // elements between batch entries (query rows of entry b start at q + b*q_bstride)
  const uint16_t* k;
  long k_ld;           // elements between consecutive keys
  long k_bstride;
  const uint16_t* v;
  long v_ld;
  long v_bstride;
  uint16_t* o;
  long o_ld;
  long o_bstride;
  int B, H, Tq, Tk;
  int head_stride;     // elements between heads (64 for [t][h*64] layouts)
};
void launch_attn_encoder(DT dt, const AttnArgs& a, hipStream_t st);
// flash attention with optional causal mask (key <= query + causal_off) and per-entry first valid key
void launch_attn_flash(DT dt, const AttnArgs& a, int causal, int causal_off, const int* kbegin, hipStream_t st);

// decoder attention (self: cache gathered through the ancestry table; cross: shared per window)
struct DecAttnArgs {
  const uint16_t* q;  // [R*Tn][q_ld]
  long q_ld;
  uint16_t* o;        // [R*Tn][d]
  int R, Tn, H, d;
  // self
  const uint16_t* kc;  // [slot][R][d]
  const uint16_t* vc;
  const int* anc;      // [R][anc_ld]  (row whose cache entry holds slot s of row r); nullptr = identity
  int anc_ld;
  const int* pad;      // [R] first valid slot
  const int* slot0;    // device scalar: slot of the first new token
  // cross
  const uint16_t* ck;  // [W][Tk][ck_ld] (k at +0, v at +d)
  long ck_ld;
  int Tk;
  int rows_per_win;    // rows sharing one encoder window (beam)
  int win_of_row_div;  // row -> window = row / rows_per_win
};
void launch_self_attn(DT dt, const DecAttnArgs& a, hipStream_t st);
// ws: cross_attn_ws_floats(H, nwin) floats for the key-split partials (nullptr = no split)
size_t cross_attn_ws_floats(int H, int nwin);
void launch_cross_attn(DT dt, const DecAttnArgs& a, float* ws, hipStream_t st);
// raw cross-attention scores of selected heads (alignment): out [nh][R*Tn][Tk] f32
void launch_cross_scores(DT dt, const DecAttnArgs& a, const int* heads_layer_local, int nh, float* out, hipStream_t st);

// weights
struct InitSpec {
  int tid;
  float scale, offset;
  long n;          // logical elements
  int kind;        // 0 plain copy order, 1 conv permute ([O][C][3] -> [O][3*C padded Kp]), 2 f32 store
  int O, C, Kp;    // conv permute
  void* dst;
  int store_f32;   // store as f32 (biases / LN) instead of 16-bit
};
void launch_init_tensor(DT dt, uint64_t seed, const InitSpec& s, hipStream_t st);

}  // namespace wmx
