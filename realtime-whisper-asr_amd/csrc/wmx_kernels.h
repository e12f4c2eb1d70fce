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
  EPI_CROSSKV = 6,     // cross K/V of all decoder layers, head-major: K [L][xw][H][kXS][64], V^T [L][xw][H][64][kXS]
  EPI_GELU_MX8 = 7,    // out8 = MX-fp8(gelu(acc + bias)): e4m3 bytes at out (ldc bytes / row), e8m0 scales at out2
  // decode step, LayerNorm folded into the projections (packed GEMM, S == 1; row_ln_from_stats):
  EPI_RESID_STATS = 8,  // x32 = out += acc + bias; out16 = 16-bit(x32); stats[n / 16][m] = (mean, M2) of x32
  EPI_LNFOLD_GELU16 = 9,  // out16 = gelu(rstd_m (acc - mean_m c1[n]) + c2[n]), (mean, rstd) from stats
  // encoder, LayerNorm folded into the projections (gemm256 only, N % 256 == 0 for the producers):
  // the residual stream is two 16-bit planes, x = out16 (hi = 16-bit(x)) + out (lo = 16-bit(x - hi)): hi is the next
  // projection's A operand, and the pair keeps ~17 significant bits through the residual adds
  EPI_RESID32_LNS = 10,     // x = hi + lo + acc + bias -> (hi, lo); stats[n / 256][m] = (mean, M2) of x's 256 columns
  EPI_GELU_POS32_LNS = 11,  // x = gelu(acc + bias) + pos[m % posT] -> (hi, lo); the same stats
  EPI_LNF_STORE16 = 12,     // out16 = rstd_m (acc - mean_m c1[n]) + bias[n], (mean, rstd) merged from stats[lng][m]
  EPI_LNF_GELU16 = 13,      // out16 = gelu(rstd_m (acc - mean_m c1[n]) + bias[n])
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
  // EPI_CROSSKV: row m = w * xt + t, column n = (l * 2 + kv) * d + h * 64 + e
  int xw = 1, xt = 1500;
  // EPI_GELU_MX8: the block scales (one byte per 32 columns, ldc2 bytes per row)
  uint8_t* out2 = nullptr;
  long ldc2 = 0;
  // EPI_RESID_STATS / EPI_LNFOLD_GELU16: row statistics [rows][stats_ld >= d / 16] (a row's 16-column groups contiguous,
  // so a consumer wave reads a row's statistics in a few lines); the 16-bit copy of x; folded constants
  float2* stats = nullptr;
  long stats_ld = 0;
  uint16_t* out16 = nullptr;
  const float* c1 = nullptr;
  const float* c2 = nullptr;
  int lng = 0;  // EPI_LNF_*: 256-column groups of the row statistics (the LayerNorm width / 256)
};

// padded key stride of the cross K/V images (a multiple of 32 keys; the pad stays zero)
constexpr int kXS = 1504;

// Cross K / V^T images of one (layer, window, head): kXS keys x 64 dims each, stored MFMA-fragment-major so that
// every wave-instruction of the decode cross attention streams one contiguous, lane-linear 1 KiB piece.
// K (A operand of S^T = K.Q^T): 32-key block kb, pair u, dim half hh, lane l = fr + 16g holds dims 32hh + 8g .. +8
//   of key 32kb + 8(fr >> 2) + 4u + (fr & 3)          -> element ((((kb*2 + u)*2 + hh)*64 + l) * 8 + j
// V^T (B operand of P.V): block kb, dim block db, lane l = fr + 16g holds keys 32kb + 8g .. +8 of dim 16db + fr
//                                                    -> element (((kb*4 + db)*64 + l) * 8 + j
// Four consecutive dims (K) or four consecutive keys (V^T) starting at a multiple of 4 are contiguous.
__host__ __device__ inline long crossk_off(int t, int c) {
  const int kb = t >> 5, tt = t & 31;
  const int u = (tt >> 2) & 1, fr = ((tt >> 3) << 2) | (tt & 3);
  const int hh = c >> 5, g = (c >> 3) & 3;
  return ((((long)kb * 2 + u) * 2 + hh) * 64 + fr + 16 * g) * 8 + (c & 7);
}
__host__ __device__ inline long crossv_off(int t, int c) {
  const int kb = t >> 5, g = (t >> 3) & 3;
  const int db = c >> 4, fr = c & 15;
  return (((long)kb * 4 + db) * 64 + fr + 16 * g) * 8 + (t & 7);
}
// byte offsets of the same elements in the fp8 images (launch_crosskv_quant): 16-bit piece P = (2 blk + hh) 64 + l
// (8 elements) sits at bytes (blk 64 + l) 16 + 8 hh
__host__ __device__ inline long crossk8_off(int t, int c) {
  const int kb = t >> 5, tt = t & 31;
  const int u = (tt >> 2) & 1, fr = ((tt >> 3) << 2) | (tt & 3);
  const int hh = c >> 5, g = (c >> 3) & 3;
  return (((long)kb * 2 + u) * 64 + fr + 16 * g) * 16 + hh * 8 + (c & 7);
}
__host__ __device__ inline long crossv8_off(int t, int c) {
  const int kb = t >> 5, g = (t >> 3) & 3;
  const int db = c >> 4, fr = c & 15;
  return (((long)kb * 2 + (db >> 1)) * 64 + fr + 16 * g) * 16 + (db & 1) * 8 + (t & 7);
}

enum GemmTile { TILE_128x128 = 0, TILE_64x64 = 1, TILE_32x64 = 2, TILE_SKINNY = 3, TILE_256 = 4 };
// K depth of one staged slice of the 256 x 256 GEMM (gemm256_kernel): 64 = the half-tile ring of whole 128-B lines
// (default, K % 64 == 0), 32 = the 32-deep slice ring (every 128-B line fetched in two halves one slice apart)
// gemm256's ring addresses a lane's rows with 32-bit element offsets (row * ld + chunk): every row base must fit
inline bool g256_offsets_fit(long M, long N, long lda, long ldw) {
  return (M - 1) * lda + 64 < (1L << 32) && (N - 1) * ldw + 64 < (1L << 32);
}
#ifndef WMX_G256_BK
#define WMX_G256_BK 64
#endif

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

// MX-fp8 GEMM (v_mfma_scale_f32_16x16x128_f8f6f4): C[M][N] = dequant(A)[M][K] . dequant(W)[N][K]^T.
// A / W: e4m3 bytes, row stride lda / ldw bytes; AS / WS: e8m0 scale bytes per 32 K (row stride ldas / ldws).
// K % 128 == 0; epilogues STORE16 / RESID32 / GELU_MX8 / STORE32 (the output dtype of STORE16 is `dt`).
struct Mx8Call {
  const uint8_t* A;
  long lda;
  const uint8_t* AS;
  long ldas;
  const uint8_t* W;
  long ldw;
  const uint8_t* WS;
  long ldws;
  int M, N, K;
  Epi epi;
};
void launch_gemm_mx8(DT dt, const Mx8Call& g, hipStream_t st);
// rows x K (bf16 / f16) -> MX-fp8 bytes [rows][K] + scales [rows][K/32] (weight preparation)
void launch_mx8_quantize_rows(DT dt, const uint16_t* src, long rows, int K, uint8_t* q, uint8_t* s, hipStream_t st);
// LayerNorm of fp32 rows straight to MX-fp8 (the A operand of the next MX-fp8 GEMM)
void launch_layernorm_mx8(const float* x, const float* g, const float* b, uint8_t* q, uint8_t* s, int rows, int d,
                          hipStream_t st);

// ---- decoder weights in MFMA-fragment-major ("packed") layout ----
// A [N][K] weight is stored as tiles of 16 rows x 32 k (1 KiB); tile (n/16, k/32) at ((n/16)*(K/32) + k/32)*512,
// inside a tile lane l = (n%16) + 16*((k%32)/8) holds k%8 = 0..7 contiguously.  One wave's B-fragment load of a
// k-step is then a single contiguous, lane-linear 1 KiB read.  Sub-matrices starting at a row multiple of 16
// (the fused QKV parts) keep the same formula with base + row0*K.  N is padded to a multiple of 16.
__host__ __device__ inline long packed_index(long n, long k, long K) {
  return (((n >> 4) * (K >> 5) + (k >> 5)) << 9) + (((n & 15) + 16 * ((k & 31) >> 3)) << 3) + (k & 7);
}
// ---- 8-bit decoder weights (model dtype WMX_DTYPE_MX8, the fp8 decode of BASELINE config 5) ----
// e4m3 bytes, one power-of-two scale per weight ROW (the OCP MX rule of mx8_exp with the block = the whole K row),
// stored as tiles of 16 rows x 64 k (1 KiB): tile (n/16, k/64) at byte ((n/16)*(K/64) + k/64)*1024; inside it lane
// l = (n%16) + 16*((k%32)/8) holds 16 bytes: k%64 in [0, 32) at bytes 0..7 and k%64 in [32, 64) at bytes 8..15
// (k%8 = 0..7 each).  One wave's 16-byte load is then the B fragments of two consecutive 32-deep MFMA k-steps,
// exactly the bf16 packed layout's lanes: the bytes are widened to the 16-bit operand in registers
// (fp8x16_to16) and the row scale multiplies the fp32 result in the epilogue.
__host__ __device__ inline long packed8_index(long n, long k, long K) {
  return (((n >> 4) * (K >> 6) + (k >> 6)) << 10) + (((n & 15) + 16 * ((k & 31) >> 3)) << 4) + (((k >> 5) & 1) << 3) +
         (k & 7);
}
// src: a packed 16-bit [N][K] matrix (packed_index) -> q8 (packed8_index, N padded to 16 rows), scale[n] = 2^e_n
// (N padded entries 0), and optionally rm = the dequantized row-major [N][K] 16-bit copy (many-row passes)
// the CTranslate2 int8 grid (model dtype I8): per-row CT2 scales (derived: 127 / max|row|, or given), int8 bytes in the
// packed8_index layout, the GEMM's row multipliers 1 / scale, and the row-major dequantized copy (rm, optional)
// shader-clock probe (bench diagnostic): n workgroups each write the MHz they ran at for `ms` of wall time
void launch_clock_probe(float* out, int n, double ms, hipStream_t st);
void launch_i8_quantize(DT dt, const uint16_t* src, int N, int K, float* ct2s, uint8_t* q8, float* mult, uint16_t* rm,
                        hipStream_t st);
void launch_w8_quantize(DT dt, const uint16_t* src, int N, int K, uint8_t* q8, float* scale, uint16_t* rm,
                        hipStream_t st);
// fp8 cross K / V^T images: per (layer, kv, window, head) image one power-of-two scale (mx8_exp of the image's
// amax); the 16-byte lane piece p = blk*64 + l of an fp8 image holds the bf16 image's pieces (2 blk + 0)*64 + l and
// (2 blk + 1)*64 + l, i.e. for K both dim halves of one key pair (u) and for V^T two dim blocks of one key block:
// one 1 KiB wave load per (32-key block, pair u) of K and per (32-key block, dim-block pair) of V^T.
// src / dst images [L*2][xw][H] of kXS*64 elements; windows [0, B) converted; scale [L*2][xw][H]
void launch_crosskv_quant(const uint16_t* src, uint8_t* dst, float* scale, int L2, int xw, int B, int H,
                          hipStream_t st);

// C[M][N] = A[M][K] . Wp^T.  S == 1: epilogue applied in-kernel.  S > 1: K is split over S workgroup slices and
// each writes raw fp32 partials part[s][M][N] (no bias); the consumer sums them in slice order (deterministic).
struct PackedCall {
  const uint16_t* A;
  long lda;
  const uint16_t* W;  // packed (packed_index), or with wscale the e4m3 bytes (packed8_index)
  int M, N, K;
  int S = 1;
  Epi epi;
  const float* wscale = nullptr;  // 8-bit weights: per-row scales (result = scale[n] * acc, before the epilogue)
  int w8kind = 1;                 // with wscale: 1 e4m3 bytes (fp8 decode), 2 int8 bytes (CTranslate2 int8 grid)
  float* part = nullptr;
  // in-situ probe: [slot][workgroup][start, end] wall-clock ticks (probe_record) at slot *pslot, or null
  unsigned long long* tprobe = nullptr;
  const int* pslot = nullptr;
  int nct = 0;  // 16-column tiles per workgroup (0: packed_nct's choice; 1, 2 or 4)
};
void launch_gemm_packed(DT dt, const PackedCall& g, hipStream_t st);
// the launch geometry launch_gemm_packed chooses: MT 16-row fragments x NCT 16-column tiles per workgroup, NW waves,
// KU k-steps of loads per batch; grid (gx column groups, S slices, gz row chunks)
struct PackedPlan {
  int MT, NCT, NW, KU, gx, gz;
};
PackedPlan packed_plan(int M, int N, int K, int S, int nct = 0, bool w8 = false);
// the element offsets a packed-GEMM lane reads, shared by gemm_packed_kernel and the host-side extent check
// (packed_extent): k-step range of one wave, the B fragment of column tile t (clamped to the last tile) and the A
// fragment of row `row` (clamped to the last row)
__host__ __device__ inline void packed_wave_ksteps(int K, int S, int NW, int sp, int wave, int& ks0, int& ks1) {
  const int ksteps = K >> 5;
  const int kps = (ksteps + S - 1) / S;
  const int kb = sp * kps, ke = min(ksteps, kb + kps);
  const int per = (max(0, ke - kb) + NW - 1) / NW;
  ks0 = kb + wave * per;
  ks1 = min(ke, ks0 + per);
}
__host__ __device__ inline long packed_w_elem(int t, int ntiles, int ksteps, int kstep, int lane) {
  return ((long)min(t, ntiles - 1) * ksteps << 9) + ((long)kstep << 9) + lane * 8;
}
__host__ __device__ inline long packed_a_elem(int row, int M, long lda, int kstep, int lane) {
  return (long)min(row, M - 1) * lda + 8 * (lane >> 4) + kstep * 32;
}
// max element offsets + 1 a launch of this shape touches: B fragments (weights), A fragments, and (S > 1) the
// fp32 partials part[s][M][N]; the k-steps any wave loads beyond its slice (must be 0)
struct PackedExtent {
  long w_end, a_end, part_end, stray_ksteps;
};
PackedExtent packed_extent(int M, int N, int K, int S, long lda, int nct = 0, bool w8 = false);
int packed_nct(int M, int N, int K);
// split count for a partial-output launch (<= cap_elems / (M*N) partial slices)
int packed_splits(int M, int N, int K, long cap_elems);

// x[m] += bias + sum_s part[s][m]; optionally out16[m] = LayerNorm(x[m]) (g == nullptr: no LN)
void launch_reduce_ln(DT dt, const float* part, int S, const float* bias, float* x, const float* g, const float* b,
                      uint16_t* out16, int rows, int d, hipStream_t st, unsigned long long* tprobe = nullptr,
                      const int* pslot = nullptr);
void gemm_init_attributes();

// log-mel
// sparse slaney filterbank limits of the FFT log-mel form (its table is staged in LDS)
constexpr int kMaxMels = 128, kMelWCap = 640;
double logmel_flops_per_frame();  // algorithmic flops of the FFT log-mel per STFT frame
// 32-frame blocks of a window of max_frames STFT frames; the statistics buffer holds B x blocks x (1 + n_mels) floats
int logmel_blocks(int max_frames);
void launch_logmel(const float* pcm, long stride, const long* lens_dev, const int* seek_dev, int B, int max_frames,
                   const int* mfirst, const int* mcount, const int* moff, const float* mw, int n_mels, float* stats,
                   long stats_cap, float* out, hipStream_t st);

// elementwise / norm / layout
void launch_layernorm(DT dt, const float* x, const float* g, const float* b, uint16_t* out, int rows, int d,
                      hipStream_t st);
// LayerNorm of residual rows held as two 16-bit planes x = hi + lo (the encoder fold's residual stream)
void launch_layernorm_split(DT dt, const uint16_t* xhi, const uint16_t* xlo, const float* g, const float* b,
                            uint16_t* out, int rows, int d, hipStream_t st);
void launch_layernorm_rows(DT dt, const float* x, const int* row_idx, const float* g, const float* b, uint16_t* out,
                           int rows, int d, hipStream_t st);
void launch_im2col_conv1(DT dt, const float* mel, int B, int n_mels, int Kp, uint16_t* out, hipStream_t st);
void launch_im2col_conv2(DT dt, const uint16_t* h1, int B, int d, uint16_t* out, hipStream_t st);
void launch_cvt16_to_f32(DT dt, const uint16_t* in, float* out, long n, hipStream_t st);
// x[r*Tn+i] = tok_emb[hist[r*hist_ld + slot]] + pos_emb[slot - pad[r]],  slot = *slot0 + i
// tok_emb is packed (packed_index), pos_emb row-major
void launch_embed(DT dt, const uint16_t* tok_emb, const uint16_t* pos_emb, const int* hist, long hist_ld, int R, int Tn,
                  const int* pad, const int* slot0, int d, float* x, hipStream_t st, int V);
// row-major [N][K] copy of a packed matrix
void launch_unpack_packed(const uint16_t* packed, uint16_t* rowmajor, int N, int K, hipStream_t st);
// decode step (Tn == 1): x = embed, out16 = LN(x) * g + b, in one launch
void launch_embed_ln(DT dt, const uint16_t* tok_emb, const uint16_t* pos_emb, const int* hist, long hist_ld, int R,
                     const int* pad, const int* slot0, const float* g, const float* b, int d, float* x, uint16_t* out,
                     hipStream_t st, int V, float2* stats = nullptr, long stats_ld = 0);
// LayerNorm (g, b) folded into the projection W (+ bias): packed Wp = W diag(g), c1 = Wp 1, c2 = bias + W b
// (rowmajor: Wp is written row-major [N][K] instead of packed: the encoder's gemm256 operand)
void launch_fold_ln(DT dt, const uint16_t* Wrm, const float* g, const float* b, const float* bias, int N, int K,
                    uint16_t* Wp, float* c1, float* c2, hipStream_t st, bool rowmajor = false);

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
  long kv_head_stride = 0;  // K/V head stride when it differs from head_stride (0: same)
  // encoder attention only: write O as MX-fp8 (bytes [row][o8_ld], scales [row][os_ld]) instead of o
  uint8_t* o8 = nullptr;
  uint8_t* os = nullptr;
  long o8_ld = 0, os_ld = 0;
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
  int kv_R;            // row stride of the KV cache ([slot][kv_R][d]); >= R
  // cross
  // cross K/V of one layer, head-major: the (window w, head h) image starts at ck / cv + w*x_wstride + h*x_hstride;
  // inside it K[t][e] sits at crossk_off(t, e) and V^T[e][t] at crossv_off(t, e) (fragment-major, see above)
  const uint16_t* ck;
  const uint16_t* cv;
  long x_wstride, x_hstride;
  int Tk;
  int rows_per_win;    // rows sharing one encoder window (beam)
  int* xcnt = nullptr; // key-chunked launches: one arrival counter per (window, head), zero between launches
  unsigned long long* tprobe = nullptr;  // [slot][workgroup][start, end] wall-clock ticks (probe_record), or null
  // decode step fed by split-K partials (qS > 0): q = bias + sum_s qpart[s*qpart_stride + m*qpart_ld + col]
  // (self attention: columns [0,d) q, [d,2d) k, [2d,3d) v; k and v are also written to the cache at slot0)
  const float* qpart = nullptr;
  int qS = 0;
  long qpart_stride = 0, qpart_ld = 0;
  const float* qbias = nullptr;
  // LayerNorm folded into the projection feeding qpart (wmx_common.h row_ln_from_stats): value =
  // rstd_row (sum_s qpart - mean_row ln_c1[col]) + ln_c2[col] instead of qbias + sum_s qpart
  const float* ln_c1 = nullptr;
  const float* ln_c2 = nullptr;
  const float2* ln_stats = nullptr;  // [rows][ln_ld >= d / 16]
  long ln_ld = 0;
  // cross attention with the query projection fused (decode, wq != null): the workgroup computes its window-rows'
  // queries of head h itself, q = qin[row] . wq[64 h .. 64 h + 63]^T + qbias, on MFMA with K split over its waves
  // (wq packed: packed_index; qin 16-bit [rows][qin_ld])
  const uint16_t* wq = nullptr;
  const uint16_t* qin = nullptr;
  long qin_ld = 0;
  const float* wq_scale = nullptr;  // wq is 8-bit (packed8_index) with these per-row scales
  // fp8 cross K / V^T images (launch_crosskv_quant layout): ck / cv point at e4m3 bytes, x_wstride / x_hstride
  // stay in elements, and the (window w, head h) image's scales are ck_scale / cv_scale[w * H + h]
  const float* ck_scale = nullptr;
  const float* cv_scale = nullptr;
  int win_of_row_div;  // row -> window = row / rows_per_win
};
void launch_self_attn(DT dt, const DecAttnArgs& a, hipStream_t st);
// ws: cross_attn_ws_floats(H, nwin, nq_max) floats for the key-chunk records (decode steps), a.xcnt: nwin*H
// zero-initialised ints (the merging workgroup re-arms its counter)
size_t cross_attn_ws_floats(int H, int nwin, int nq_max);
void launch_cross_attn(DT dt, const DecAttnArgs& a, float* ws, hipStream_t st);
// raw cross-attention scores of selected heads (alignment): out [nh][R*Tn][Tk] f32
void launch_cross_scores(DT dt, const DecAttnArgs& a, const int* heads_layer_local, int nh, float* out, hipStream_t st);

// pre-ASR DSP (wmx_dsp.hip)
constexpr int kMaxTaps = 17;      // filtfilt: up to an order-16 transfer function
constexpr int kDedupMaxN = 8000;  // dedup features: samples per chunk (0.5 s at 16 kHz)
struct IIRCoefs {
  double b[kMaxTaps], a[kMaxTaps], zi[kMaxTaps - 1];
  int ntaps, padlen;
};
void launch_filtfilt(const float* x, long xstride, const long* lens_dev, int B, const IIRCoefs& f, double* scratch,
                     long sstride, float* y, long ystride, hipStream_t st);
void launch_dedup_features(const float* x, long xstride, const long* lens_dev, int B, float sr, float* feats,
                           hipStream_t st);

// Silero VAD v5, 16 kHz (wmx_vad.hip): f32 weight image, offsets in floats.  The LSTM matrices are stored
// transposed ([128][512]) so a gate-per-thread read is one contiguous row per k.
constexpr int kVadWindow = 512, kVadContext = 64, kVadInput = 576, kVadPadded = 640, kVadHidden = 128;
constexpr long kVadOffBasis = 0;
constexpr long kVadOffC0w = kVadOffBasis + 258L * 256, kVadOffC0b = kVadOffC0w + 128L * 129 * 3;
constexpr long kVadOffC1w = kVadOffC0b + 128, kVadOffC1b = kVadOffC1w + 64L * 128 * 3;
constexpr long kVadOffC2w = kVadOffC1b + 64, kVadOffC2b = kVadOffC2w + 64L * 64 * 3;
constexpr long kVadOffC3w = kVadOffC2b + 64, kVadOffC3b = kVadOffC3w + 128L * 64 * 3;
constexpr long kVadOffWihT = kVadOffC3b + 128, kVadOffWhhT = kVadOffWihT + 512L * 128;
constexpr long kVadOffBih = kVadOffWhhT + 512L * 128, kVadOffBhh = kVadOffBih + 512;
constexpr long kVadOffW2 = kVadOffBhh + 512, kVadOffB2 = kVadOffW2 + 128;
constexpr long kVadWeights = kVadOffB2 + 1;
void launch_vad(const float* W, const float* pcm, long stride, float* ctx, float* state, const int* slots_dev, int S,
                int nwin, float* enc, float* probs, hipStream_t st);

// weights
struct InitSpec {
  int tid;
  float scale, offset;
  long n;          // logical elements
  int kind;        // 0 plain copy order, 1 conv permute ([O][C][3] -> [O][3*C padded Kp]), 2 packed [O][Kp]
  int O, C, Kp;    // conv permute / packed (Kp = K)
  void* dst;
  int store_f32;   // store as f32 (biases / LN) instead of 16-bit
};
void launch_init_tensor(DT dt, uint64_t seed, const InitSpec& s, hipStream_t st);

}  // namespace wmx
