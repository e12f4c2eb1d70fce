// libwmx runtime: model weight arena, per-context buffers, the transcribe pipeline and the C ABI (include/wmx.h).
//
// Pipeline (SURVEY.md §3 stack C, re-designed for one MI355X):
//   pcm (HBM) -> log-mel (f32 MFMA DFT) -> encoder (bf16/f16 MFMA GEMMs, flash attention, fp32 residual)
//   -> cross K/V of every decoder layer in ONE GEMM (once per window, shared by all beams)
//   -> [language detect: one decoder step on <|startoftranscript|>]
//   -> prompt prefill (left-padded so all windows advance in lock-step; beams alias beam 0's prompt cache
//      through the ancestry table) -> decode loop, one step = one hipGraph replay, state entirely on device
//   -> [alignment forward over sot + text + eot: alignment-head scores -> softmax/normalise/median on device,
//      DTW on host threads].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/wmx_diag.h"  // (includes wmx.h)
#include "wmx_common.h"
#include "wmx_decode.h"
#include "wmx_kernels.h"

namespace wmx {

static thread_local std::string g_err;

// ------------------------------------------------------------------------------------------------
// host helpers
// ------------------------------------------------------------------------------------------------
static uint16_t host_f32_to_bf16(float f) { return f32_to_bf16(f); }
static uint16_t host_f32_to_f16(float f) {
  _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}
static float host_bf16_to_f32(uint16_t h) { return bf16_to_f32(h); }
static float host_f16_to_f32(uint16_t u) {
  _Float16 h;
  std::memcpy(&h, &u, 2);
  return (float)h;
}

// faster-whisper FeatureExtractor.get_mel_filters (slaney), evaluated in double
static std::vector<double> mel_filters(int n_mels) {
  const int nb = 201;
  std::vector<double> fft(nb), mels(n_mels + 2), freqs(n_mels + 2);
  for (int i = 0; i < nb; ++i) fft[i] = i * 16000.0 / 400.0;
  for (int i = 0; i < n_mels + 2; ++i) mels[i] = 45.245640471924965 * i / (n_mels + 1);
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  for (int i = 0; i < n_mels + 2; ++i)
    freqs[i] = mels[i] >= min_log_mel ? min_log_hz * std::exp(logstep * (mels[i] - min_log_mel)) : f_sp * mels[i];
  std::vector<double> w((size_t)n_mels * nb);
  for (int m = 0; m < n_mels; ++m) {
    const double enorm = 2.0 / (freqs[m + 2] - freqs[m]);
    for (int k = 0; k < nb; ++k) {
      const double lower = -(freqs[m] - fft[k]) / (freqs[m + 1] - freqs[m]);
      const double upper = (freqs[m + 2] - fft[k]) / (freqs[m + 2] - freqs[m + 1]);
      w[(size_t)m * nb + k] = std::max(0.0, std::min(lower, upper)) * enorm;
    }
  }
  return w;
}

static std::vector<float> sinusoids(int length, int channels) {
  std::vector<float> out((size_t)length * channels);
  const int half = channels / 2;
  const double inc = std::log(10000.0) / (half - 1);
  for (int t = 0; t < length; ++t)
    for (int i = 0; i < half; ++i) {
      const double v = t * std::exp(-inc * i);
      out[(size_t)t * channels + i] = (float)std::sin(v);
      out[(size_t)t * channels + half + i] = (float)std::cos(v);
    }
  return out;
}

struct Special {
  int eot = 50257, sot = 50258, lang0 = 50259, n_langs, translate, transcribe, sot_lm, sot_prev, no_speech,
      no_timestamps, timestamp_begin, blank = 220;
  explicit Special(int n_vocab) {
    n_langs = n_vocab >= 51866 ? 100 : 99;
    const int base = 50259 + n_langs;
    translate = base;
    transcribe = base + 1;
    sot_lm = base + 2;
    sot_prev = base + 3;
    no_speech = base + 4;
    no_timestamps = base + 5;
    timestamp_begin = base + 6;
  }
};

// ------------------------------------------------------------------------------------------------
// model
// ------------------------------------------------------------------------------------------------
struct TensorEntry {
  std::string name;
  int tid;
  long n;           // logical elements
  float scale, offset;
  int kind;         // 0 plain, 1 conv permute
  int C, Kp, O;
  void* dst;
  int store_f32;
  std::vector<long> shape;
};

struct EncLayer {
  float *ln1g, *ln1b, *bqkv, *bo, *ln2g, *ln2b, *bfc1, *bfc2;
  uint16_t *wqkv, *wo, *wfc1, *wfc2;
  // MX-fp8 copies of the four projections (model dtype WMX_DTYPE_MX8): e4m3 [N][K] + e8m0 scales [N][K/32]
  uint8_t *qkv8 = nullptr, *qkv8s = nullptr, *o8 = nullptr, *o8s = nullptr, *fc18 = nullptr, *fc18s = nullptr,
          *fc28 = nullptr, *fc28s = nullptr;
  // LayerNorm folded into qkv (LN1) and fc1 (LN2) (Model::enc_fold): row-major W diag(g), c1 = W' 1, c2 = bias + W b
  uint16_t *fqkv = nullptr, *ffc1 = nullptr;
  float *c1qkv = nullptr, *c2qkv = nullptr, *c1fc1 = nullptr, *c2fc1 = nullptr;
};
struct DecLayer {
  float *ln1g, *ln1b, *bqkv, *bo, *ln2g, *ln2b, *bcq, *bco, *ln3g, *ln3b, *bfc1, *bfc2;
  uint16_t *wqkv, *wo, *wcq, *wco, *wfc1, *wfc2;
  // row-major [N][K] copies of the packed projections (derived after every weight load) for the many-row
  // passes (prompt prefill, word-alignment forward), which run on the tiled MFMA GEMM instead of the packed one
  uint16_t *rqkv, *ro, *rcq, *rco, *rfc1, *rfc2;
  // the decode step's LayerNorm-folded projections (wmx_common.h row_ln_from_stats; derived after every weight
  // load): packed W diag(g) of qkv (LN1), cross-q (LN2), fc1 (LN3) and their c1 = W' 1, c2 = bias + W b
  uint16_t *fqkv, *fcq, *ffc1;
  float *c1qkv, *c2qkv, *c1cq, *c2cq, *c1fc1, *c2fc1;
  // fp8 decode (Model::w8): e4m3 copies of the six packed projections (packed8_index) + per-row scales, derived
  // after every weight load (launch_w8_quantize); the row-major copies above then hold their dequantized values
  uint8_t *q8qkv = nullptr, *q8o = nullptr, *q8cq = nullptr, *q8co = nullptr, *q8fc1 = nullptr, *q8fc2 = nullptr;
  float *s8qkv = nullptr, *s8o = nullptr, *s8cq = nullptr, *s8co = nullptr, *s8fc1 = nullptr, *s8fc2 = nullptr;
  // the CTranslate2 int8 grid (Model::i8): the CT2 per-row scales of the six projections (parameters: a CT2 int8
  // checkpoint's weight_scale, or derived by CT2's rule 127 / max|row|); q8* then hold int8 bytes and s8* 1 / scale
  float *i8sqkv = nullptr, *i8so = nullptr, *i8scq = nullptr, *i8sco = nullptr, *i8sfc1 = nullptr, *i8sfc2 = nullptr;
};

struct Model {
  wmx_dims d{};
  int device = 0;
  DT dt = DT::BF16;
  bool mx8 = false;  // encoder projections on MX-fp8 MFMA (BASELINE config 5); everything else in `dt`
  // fp8 decode (model dtype MX8 unless WMX_DEC_FP8=0): the decoder projections and the logits projection on 8-bit
  // weights (DecLayer::q8*, tok8), the cross K / V images in fp8 (Ctx::ckv8); the embedding lookup, LayerNorms,
  // biases, the self-attention KV cache and all activations stay 16-bit / fp32
  bool w8 = false;
  uint8_t* tok8 = nullptr;  // the token embedding as the logits projection's 8-bit weights (packed8_index)
  float* tok8s = nullptr;
  // the CTranslate2 int8 grid (model dtypes WMX_DTYPE_I8 / I8_BF16, the reference's int8_float16 / int8): the 8-bit
  // decode path with int8 bytes and CT2's per-row scales instead of e4m3 (w8 is set too); the cross K / V images stay
  // 16-bit (kv8 false) and the cross-q projection runs as its own launch on the int8 weights (no fused 8-bit form);
  // the encoder and the cross-K/V projection run on the 16-bit weights (a CT2 int8 checkpoint's dequantized q / s)
  bool i8 = false;
  bool kv8 = false;  // the fp8 cross K / V images (the MX8 model's fp8 decode)
  float* i8stok = nullptr;  // CT2 scales of the token embedding (the logits projection)
  std::map<std::string, std::pair<float*, long>> i8_scale_dst;  // weight name -> (its scale rows, row count)
  size_t param_bytes = 0;  // the arena's parameter region [0, param_bytes): what a weight broadcast must carry
  std::vector<std::pair<size_t, size_t>> guards;  // debug guard gaps (WMX_GUARD), Planner::guards
  char* arena = nullptr;
  size_t arena_bytes = 0;
  int K1p = 0;
  uint16_t *conv1w = nullptr, *conv2w = nullptr, *tok_emb = nullptr, *dec_pos = nullptr, *wckv = nullptr;
  float *conv1b = nullptr, *conv2b = nullptr, *enc_pos = nullptr, *lnpg = nullptr, *lnpb = nullptr, *bckv = nullptr,
        *lng = nullptr, *lnb = nullptr;
  std::vector<EncLayer> enc;
  std::vector<DecLayer> dec;
  std::vector<TensorEntry> entries;
  std::map<std::string, int> by_name;
  // log-mel constants
  int *mel_first = nullptr, *mel_count = nullptr, *mel_off = nullptr;
  float* mel_w = nullptr;
  bool initialized = false;
  bool dirty = false;  // a tensor was set since the derived copies (row-major, MX-fp8, folded) were made
  bool fold = false;   // decode step on the LayerNorm-folded projections (WMX_FOLD=1; default: reduce_ln form)
  // the mixed decode step (dec_step_mixed): the d x d residual producers (out-proj, cross-out) unsplit with row
  // statistics and LN2 / LN3 folded into their consumers (the fused cross-q projection, fc1); fc2 stays split-K +
  // reduce_ln.  16-bit models only (the fp8 decode keeps the fast step)
  // encoder: the two LayerNorms of every layer folded into qkv / fc1 (the residual producers leave x's 16-bit copy
  // and per-256-column statistics); 16-bit models with a width multiple of 256 (WMX_ENC_FOLD=0 turns it off)
  bool enc_fold = false;
  bool mixed = false;
  hipStream_t st = nullptr;
};

struct Planner {
  size_t off = 0;
  std::vector<std::pair<void**, size_t>> items;
  // debug (WMX_GUARD=1 at model / context creation): a guard gap after every buffer, filled with a byte pattern and
  // checked by wmx_debug_guard_check -- an out-of-bounds write names the buffer it ran past
  size_t guard = 0;
  std::vector<std::pair<size_t, size_t>> guards;  // (offset, bytes) of each buffer's trailing gap, in add order
  template <class T>
  void add(T** p, size_t elems) {
    items.push_back({(void**)p, off});
    off += (elems * sizeof(T) + 255) / 256 * 256;
    if (guard) {
      guards.push_back({off, guard});
      off += guard;
    }
  }
  void bind(char* base) {
    for (auto& it : items) *it.first = base + it.second;
  }
};

static void build_model(Model& m) {
  const wmx_dims& d = m.d;
  const int da = d.n_audio_state, dt = d.n_text_state, M = d.n_mels, V = d.n_vocab;
  WMX_CHECK(da % 64 == 0 && dt % 64 == 0 && da / 64 == d.n_audio_head && dt / 64 == d.n_text_head,
            "model: head_dim must be 64 and width a multiple of 64");
  WMX_CHECK(d.n_audio_ctx == 1500 && d.n_text_ctx <= 448 && M <= 128, "model: unsupported context sizes");
  m.K1p = (3 * M + 63) / 64 * 64;
  // the parameter region first (every TensorEntry destination: what a checkpoint or a weight broadcast fills),
  // then everything derived from it on each rank (positions, MX-fp8 / folded / row-major / 8-bit copies, log-mel
  // constants), so a broadcast of [0, param_bytes) is all a rank needs before wmx_model_arena_loaded
  Planner P;
  P.guard = getenv("WMX_GUARD") ? 65536 : 0;
  P.add(&m.conv1w, (size_t)da * m.K1p);
  P.add(&m.conv1b, da);
  P.add(&m.conv2w, (size_t)da * 3 * da);
  P.add(&m.conv2b, da);
  m.enc.resize(d.n_audio_layer);
  for (auto& L : m.enc) {
    P.add(&L.ln1g, da);
    P.add(&L.ln1b, da);
    P.add(&L.wqkv, (size_t)3 * da * da);
    P.add(&L.bqkv, 3 * da);
    P.add(&L.wo, (size_t)da * da);
    P.add(&L.bo, da);
    P.add(&L.ln2g, da);
    P.add(&L.ln2b, da);
    P.add(&L.wfc1, (size_t)4 * da * da);
    P.add(&L.bfc1, 4 * da);
    P.add(&L.wfc2, (size_t)4 * da * da);
    P.add(&L.bfc2, da);
  }
  P.add(&m.lnpg, da);
  P.add(&m.lnpb, da);
  const int Vp = (V + 15) / 16 * 16;
  P.add(&m.tok_emb, (size_t)Vp * dt);  // packed: rows padded to a 16-row tile
  P.add(&m.dec_pos, (size_t)d.n_text_ctx * dt);
  m.dec.resize(d.n_text_layer);
  for (auto& L : m.dec) {
    P.add(&L.ln1g, dt);
    P.add(&L.ln1b, dt);
    P.add(&L.wqkv, (size_t)3 * dt * dt);
    P.add(&L.bqkv, 3 * dt);
    P.add(&L.wo, (size_t)dt * dt);
    P.add(&L.bo, dt);
    P.add(&L.ln2g, dt);
    P.add(&L.ln2b, dt);
    P.add(&L.wcq, (size_t)dt * dt);
    P.add(&L.bcq, dt);
    P.add(&L.wco, (size_t)dt * dt);
    P.add(&L.bco, dt);
    P.add(&L.ln3g, dt);
    P.add(&L.ln3b, dt);
    P.add(&L.wfc1, (size_t)4 * dt * dt);
    P.add(&L.bfc1, 4 * dt);
    P.add(&L.wfc2, (size_t)4 * dt * dt);
    P.add(&L.bfc2, dt);
  }
  P.add(&m.wckv, (size_t)d.n_text_layer * 2 * dt * dt);
  P.add(&m.bckv, (size_t)d.n_text_layer * 2 * dt);
  P.add(&m.lng, dt);
  P.add(&m.lnb, dt);
  P.add(&m.enc_pos, (size_t)1500 * da);  // (settable: encoder.embed_positions.weight)
  if (m.i8) {  // CT2 row scales: parameters (a CT2 int8 checkpoint sets them; a broadcast carries them)
    for (auto& L : m.dec) {
      P.add(&L.i8sqkv, (size_t)3 * dt);
      P.add(&L.i8so, dt);
      P.add(&L.i8scq, dt);
      P.add(&L.i8sco, dt);
      P.add(&L.i8sfc1, (size_t)4 * dt);
      P.add(&L.i8sfc2, dt);
    }
    P.add(&m.i8stok, (size_t)(V + 15) / 16 * 16);
  }
  m.param_bytes = P.off;
  // ---- derived on every rank ----
  if (m.mx8) {
    WMX_CHECK(da % 128 == 0, "model: MX-fp8 encoder needs a width multiple of 128");
    for (auto& L : m.enc) {
      P.add(&L.qkv8, (size_t)3 * da * da);
      P.add(&L.qkv8s, (size_t)3 * da * da / 32);
      P.add(&L.o8, (size_t)da * da);
      P.add(&L.o8s, (size_t)da * da / 32);
      P.add(&L.fc18, (size_t)4 * da * da);
      P.add(&L.fc18s, (size_t)4 * da * da / 32);
      P.add(&L.fc28, (size_t)4 * da * da);
      P.add(&L.fc28s, (size_t)4 * da * da / 32);
    }
  }
  for (auto& L : m.enc) {
    if (!m.enc_fold) break;
    P.add(&L.fqkv, (size_t)3 * da * da);
    P.add(&L.ffc1, (size_t)4 * da * da);
    P.add(&L.c1qkv, 3 * da);
    P.add(&L.c2qkv, 3 * da);
    P.add(&L.c1fc1, 4 * da);
    P.add(&L.c2fc1, 4 * da);
  }
  for (auto& L : m.dec) {
    if (!m.mixed) break;  // the folded copies exist only for the mixed step
    P.add(&L.fqkv, (size_t)3 * dt * dt);
    P.add(&L.fcq, (size_t)dt * dt);
    P.add(&L.ffc1, (size_t)4 * dt * dt);
    P.add(&L.c1qkv, 3 * dt);
    P.add(&L.c2qkv, 3 * dt);
    P.add(&L.c1cq, dt);
    P.add(&L.c2cq, dt);
    P.add(&L.c1fc1, 4 * dt);
    P.add(&L.c2fc1, 4 * dt);
  }
  for (auto& L : m.dec) {
    P.add(&L.rqkv, (size_t)3 * dt * dt);
    P.add(&L.ro, (size_t)dt * dt);
    P.add(&L.rcq, (size_t)dt * dt);
    P.add(&L.rco, (size_t)dt * dt);
    P.add(&L.rfc1, (size_t)4 * dt * dt);
    P.add(&L.rfc2, (size_t)4 * dt * dt);
  }
  if (m.w8) {
    WMX_CHECK(dt % 64 == 0, "model: the fp8 decode needs a text width multiple of 64");
    for (auto& L : m.dec) {
      P.add(&L.q8qkv, (size_t)3 * dt * dt);
      P.add(&L.s8qkv, (size_t)3 * dt);
      P.add(&L.q8o, (size_t)dt * dt);
      P.add(&L.s8o, (size_t)dt);
      P.add(&L.q8cq, (size_t)dt * dt);
      P.add(&L.s8cq, (size_t)dt);
      P.add(&L.q8co, (size_t)dt * dt);
      P.add(&L.s8co, (size_t)dt);
      P.add(&L.q8fc1, (size_t)4 * dt * dt);
      P.add(&L.s8fc1, (size_t)4 * dt);
      P.add(&L.q8fc2, (size_t)4 * dt * dt);
      P.add(&L.s8fc2, (size_t)dt);
    }
    P.add(&m.tok8, (size_t)Vp * dt);
    P.add(&m.tok8s, (size_t)Vp);
  }
  // log-mel constants
  P.add(&m.mel_first, M);
  P.add(&m.mel_count, M);
  P.add(&m.mel_off, M);
  P.add(&m.mel_w, (size_t)M * 201);
  m.arena_bytes = P.off;
  WMX_HIP(hipMalloc(&m.arena, m.arena_bytes));
  WMX_HIP(hipMemsetAsync(m.arena, 0, m.arena_bytes, m.st));
  for (const auto& g : P.guards) WMX_HIP(hipMemsetAsync(m.arena + g.first, 0xA5, g.second, m.st));
  m.guards = P.guards;
  P.bind(m.arena);

  // tensor registry, in oracle/whisper_np.py tensor_specs order (tid = index)
  auto f32s = [](double v) { return (float)v; };
  auto add = [&](const std::string& name, std::vector<long> shape, float scale, float offset, void* dst, int store_f32,
                 int kind = 0, int C = 0, int Kp = 0) {
    TensorEntry e;
    e.name = name;
    e.tid = (int)m.entries.size();
    e.n = 1;
    for (long s : shape) e.n *= s;
    e.shape = shape;
    e.scale = scale;
    e.offset = offset;
    e.kind = kind;
    e.C = C;
    e.Kp = Kp;
    e.O = (int)shape[0];
    e.dst = dst;
    e.store_f32 = store_f32;
    m.by_name[name] = (int)m.entries.size();
    m.entries.push_back(e);
  };
  auto lin = [&](const std::string& p, long n_out, long n_in, uint16_t* w, float* b, bool packed = false) {
    // decoder projections are stored packed (MFMA-fragment-major, see packed_index)
    add(p + ".weight", {n_out, n_in}, f32s(1.0 / std::sqrt((double)n_in)), 0.f, w, 0, packed ? 2 : 0, 0,
        packed ? (int)n_in : 0);
    if (b) add(p + ".bias", {n_out}, 0.02f, 0.f, b, 1);
  };
  auto ln = [&](const std::string& p, long n, float* g, float* b) {
    add(p + ".weight", {n}, 0.1f, 1.0f, g, 1);
    add(p + ".bias", {n}, 0.02f, 0.f, b, 1);
  };
  add("encoder.conv1.weight", {da, M, 3}, f32s(1.0 / std::sqrt(3.0 * M)), 0.f, m.conv1w, 0, 1, M, m.K1p);
  add("encoder.conv1.bias", {da}, 0.02f, 0.f, m.conv1b, 1);
  add("encoder.conv2.weight", {da, da, 3}, f32s(1.0 / std::sqrt(3.0 * da)), 0.f, m.conv2w, 0, 1, da, 3 * da);
  add("encoder.conv2.bias", {da}, 0.02f, 0.f, m.conv2b, 1);
  for (int i = 0; i < d.n_audio_layer; ++i) {
    EncLayer& L = m.enc[i];
    const std::string p = "encoder.layers." + std::to_string(i);
    ln(p + ".self_attn_layer_norm", da, L.ln1g, L.ln1b);
    lin(p + ".self_attn.q_proj", da, da, L.wqkv, L.bqkv);
    lin(p + ".self_attn.k_proj", da, da, L.wqkv + (size_t)da * da, nullptr);
    lin(p + ".self_attn.v_proj", da, da, L.wqkv + (size_t)2 * da * da, L.bqkv + 2 * da);
    lin(p + ".self_attn.out_proj", da, da, L.wo, L.bo);
    ln(p + ".final_layer_norm", da, L.ln2g, L.ln2b);
    lin(p + ".fc1", 4 * da, da, L.wfc1, L.bfc1);
    lin(p + ".fc2", da, 4 * da, L.wfc2, L.bfc2);
  }
  ln("encoder.layer_norm", da, m.lnpg, m.lnpb);
  add("decoder.embed_tokens.weight", {V, dt}, f32s(6.0 / std::sqrt((double)dt)), 0.f, m.tok_emb, 0, 2, 0, dt);
  add("decoder.embed_positions.weight", {d.n_text_ctx, dt}, 0.05f, 0.f, m.dec_pos, 0);
  for (int i = 0; i < d.n_text_layer; ++i) {
    DecLayer& L = m.dec[i];
    const std::string p = "decoder.layers." + std::to_string(i);
    ln(p + ".self_attn_layer_norm", dt, L.ln1g, L.ln1b);
    lin(p + ".self_attn.q_proj", dt, dt, L.wqkv, L.bqkv, true);
    lin(p + ".self_attn.k_proj", dt, dt, L.wqkv + (size_t)dt * dt, nullptr, true);
    lin(p + ".self_attn.v_proj", dt, dt, L.wqkv + (size_t)2 * dt * dt, L.bqkv + 2 * dt, true);
    lin(p + ".self_attn.out_proj", dt, dt, L.wo, L.bo, true);
    ln(p + ".encoder_attn_layer_norm", dt, L.ln2g, L.ln2b);
    lin(p + ".encoder_attn.q_proj", dt, dt, L.wcq, L.bcq, true);
    lin(p + ".encoder_attn.k_proj", dt, dt, m.wckv + (size_t)i * 2 * dt * dt, nullptr);
    lin(p + ".encoder_attn.v_proj", dt, dt, m.wckv + ((size_t)i * 2 * dt + dt) * dt, m.bckv + (size_t)i * 2 * dt + dt);
    lin(p + ".encoder_attn.out_proj", dt, dt, L.wco, L.bco, true);
    ln(p + ".final_layer_norm", dt, L.ln3g, L.ln3b);
    lin(p + ".fc1", 4 * dt, dt, L.wfc1, L.bfc1, true);
    lin(p + ".fc2", dt, 4 * dt, L.wfc2, L.bfc2, true);
  }
  ln("decoder.layer_norm", dt, m.lng, m.lnb);
  if (m.i8) {  // weight name -> its CT2 row scales (wmx_model_set_row_scales)
    m.i8_scale_dst["decoder.embed_tokens.weight"] = {m.i8stok, V};
    for (int i = 0; i < d.n_text_layer; ++i) {
      DecLayer& L = m.dec[i];
      const std::string p = "decoder.layers." + std::to_string(i);
      m.i8_scale_dst[p + ".self_attn.q_proj.weight"] = {L.i8sqkv, dt};
      m.i8_scale_dst[p + ".self_attn.k_proj.weight"] = {L.i8sqkv + dt, dt};
      m.i8_scale_dst[p + ".self_attn.v_proj.weight"] = {L.i8sqkv + 2 * dt, dt};
      m.i8_scale_dst[p + ".self_attn.out_proj.weight"] = {L.i8so, dt};
      m.i8_scale_dst[p + ".encoder_attn.q_proj.weight"] = {L.i8scq, dt};
      m.i8_scale_dst[p + ".encoder_attn.out_proj.weight"] = {L.i8sco, dt};
      m.i8_scale_dst[p + ".fc1.weight"] = {L.i8sfc1, 4 * dt};
      m.i8_scale_dst[p + ".fc2.weight"] = {L.i8sfc2, dt};
    }
  }

  // constants: sinusoids, sparse mel filterbank
  auto pos = sinusoids(1500, da);
  WMX_HIP(hipMemcpyAsync(m.enc_pos, pos.data(), pos.size() * 4, hipMemcpyHostToDevice, m.st));
  auto fw = mel_filters(M);
  std::vector<int> first(M), count(M), off(M);
  std::vector<float> wts;
  for (int i = 0; i < M; ++i) {
    int lo = -1, hi = -1;
    for (int k = 0; k < 201; ++k)
      if (fw[(size_t)i * 201 + k] > 0) {
        if (lo < 0) lo = k;
        hi = k;
      }
    if (lo < 0) lo = hi = 0;
    first[i] = lo;
    count[i] = hi - lo + 1;
    off[i] = (int)wts.size();
    for (int k = lo; k <= hi; ++k) wts.push_back((float)fw[(size_t)i * 201 + k]);
  }
  WMX_HIP(hipMemcpyAsync(m.mel_first, first.data(), M * 4, hipMemcpyHostToDevice, m.st));
  WMX_HIP(hipMemcpyAsync(m.mel_count, count.data(), M * 4, hipMemcpyHostToDevice, m.st));
  WMX_HIP(hipMemcpyAsync(m.mel_off, off.data(), M * 4, hipMemcpyHostToDevice, m.st));
  WMX_CHECK(M <= kMaxMels && wts.size() <= (size_t)kMelWCap && (size_t)M * 201 >= (size_t)kMelWCap,
            "mel filterbank exceeds the log-mel kernel's LDS table");
  WMX_HIP(hipMemcpyAsync(m.mel_w, wts.data(), wts.size() * 4, hipMemcpyHostToDevice, m.st));
  WMX_HIP(hipStreamSynchronize(m.st));
}

// row-major copies of the packed decoder projections (after every weight load; deterministic)
static void prepare_rowmajor(Model& m) {
  const int dt = m.d.n_text_state;
  for (auto& L : m.dec) {
    launch_unpack_packed(L.wqkv, L.rqkv, 3 * dt, dt, m.st);
    launch_unpack_packed(L.wo, L.ro, dt, dt, m.st);
    launch_unpack_packed(L.wcq, L.rcq, dt, dt, m.st);
    launch_unpack_packed(L.wco, L.rco, dt, dt, m.st);
    launch_unpack_packed(L.wfc1, L.rfc1, 4 * dt, dt, m.st);
    launch_unpack_packed(L.wfc2, L.rfc2, dt, 4 * dt, m.st);
  }
  WMX_HIP(hipStreamSynchronize(m.st));
}

// MX-fp8 mode: derive the e4m3 + e8m0 copies of the encoder projections from the 16-bit weights (after every
// weight load; deterministic, so ranks that receive the broadcast arena may redo it harmlessly)
// WMX_DEBUG_SYNC=1: after a preparation stage, wait for the device, give an asynchronous fault time to be delivered
// and report it under the stage's name
static void debug_device(const char* what) {
  static const bool on = getenv("WMX_DEBUG_SYNC") != nullptr;
  if (!on) return;
  hipError_t e = hipDeviceSynchronize();
  usleep(300000);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipGetLastError();
  fprintf(stderr, "[wmx debug] %s: %s\n", what, hipGetErrorString(e));
  if (e != hipSuccess) throw std::runtime_error(std::string("debug check after ") + what + ": " + hipGetErrorString(e));
}

static void prepare_fold(Model& m) {
  if (m.enc_fold) {
    const int da = m.d.n_audio_state;
    for (auto& L : m.enc) {
      launch_fold_ln(m.dt, L.wqkv, L.ln1g, L.ln1b, L.bqkv, 3 * da, da, L.fqkv, L.c1qkv, L.c2qkv, m.st, true);
      launch_fold_ln(m.dt, L.wfc1, L.ln2g, L.ln2b, L.bfc1, 4 * da, da, L.ffc1, L.c1fc1, L.c2fc1, m.st, true);
    }
    WMX_HIP(hipStreamSynchronize(m.st));
  }
  if (!m.mixed) return;
  const int dt = m.d.n_text_state;
  for (auto& L : m.dec) {
    launch_fold_ln(m.dt, L.rqkv, L.ln1g, L.ln1b, L.bqkv, 3 * dt, dt, L.fqkv, L.c1qkv, L.c2qkv, m.st);
    launch_fold_ln(m.dt, L.rcq, L.ln2g, L.ln2b, L.bcq, dt, dt, L.fcq, L.c1cq, L.c2cq, m.st);
    launch_fold_ln(m.dt, L.rfc1, L.ln3g, L.ln3b, L.bfc1, 4 * dt, dt, L.ffc1, L.c1fc1, L.c2fc1, m.st);
  }
  WMX_HIP(hipStreamSynchronize(m.st));
}

static void prepare_mx8(Model& m) {
  if (!m.mx8) return;
  const int da = m.d.n_audio_state;
  for (auto& L : m.enc) {
    launch_mx8_quantize_rows(m.dt, L.wqkv, 3L * da, da, L.qkv8, L.qkv8s, m.st);
    launch_mx8_quantize_rows(m.dt, L.wo, da, da, L.o8, L.o8s, m.st);
    launch_mx8_quantize_rows(m.dt, L.wfc1, 4L * da, da, L.fc18, L.fc18s, m.st);
    launch_mx8_quantize_rows(m.dt, L.wfc2, da, 4 * da, L.fc28, L.fc28s, m.st);
  }
  WMX_HIP(hipStreamSynchronize(m.st));
}

// fp8 decode: the 8-bit copies of the decoder projections and of the logits projection (the token embedding), and
// the row-major copies overwritten with the dequantized weights, so that the many-row passes (prefill, alignment)
// run the same model as the decode step (after prepare_rowmajor; deterministic)
static void prepare_w8(Model& m) {
  if (!m.w8) return;
  const int dt = m.d.n_text_state;
  if (m.i8) {
    // the CTranslate2 int8 grid: int8 bytes with CT2's row scales.  A row's scale is given (a CT2 checkpoint's
    // weight_scale, wmx_model_set_row_scales) when its entry is > 0, else derived by CT2's rule and stored; a weight
    // set after its scales zeroes them (wmx_model_set_tensor).  The state is the scale array itself, in the
    // broadcast parameter region, so every rank of a weight broadcast derives nothing the sender did not.
    for (DecLayer& L : m.dec) {
      launch_i8_quantize(m.dt, L.wqkv, 3 * dt, dt, L.i8sqkv, L.q8qkv, L.s8qkv, L.rqkv, m.st);
      launch_i8_quantize(m.dt, L.wo, dt, dt, L.i8so, L.q8o, L.s8o, L.ro, m.st);
      launch_i8_quantize(m.dt, L.wcq, dt, dt, L.i8scq, L.q8cq, L.s8cq, L.rcq, m.st);
      launch_i8_quantize(m.dt, L.wco, dt, dt, L.i8sco, L.q8co, L.s8co, L.rco, m.st);
      launch_i8_quantize(m.dt, L.wfc1, 4 * dt, dt, L.i8sfc1, L.q8fc1, L.s8fc1, L.rfc1, m.st);
      launch_i8_quantize(m.dt, L.wfc2, dt, 4 * dt, L.i8sfc2, L.q8fc2, L.s8fc2, L.rfc2, m.st);
    }
    launch_i8_quantize(m.dt, m.tok_emb, m.d.n_vocab, dt, m.i8stok, m.tok8, m.tok8s, nullptr, m.st);
    WMX_HIP(hipStreamSynchronize(m.st));
    return;
  }
  for (auto& L : m.dec) {
    launch_w8_quantize(m.dt, L.wqkv, 3 * dt, dt, L.q8qkv, L.s8qkv, L.rqkv, m.st);
    launch_w8_quantize(m.dt, L.wo, dt, dt, L.q8o, L.s8o, L.ro, m.st);
    launch_w8_quantize(m.dt, L.wcq, dt, dt, L.q8cq, L.s8cq, L.rcq, m.st);
    launch_w8_quantize(m.dt, L.wco, dt, dt, L.q8co, L.s8co, L.rco, m.st);
    launch_w8_quantize(m.dt, L.wfc1, 4 * dt, dt, L.q8fc1, L.s8fc1, L.rfc1, m.st);
    launch_w8_quantize(m.dt, L.wfc2, dt, 4 * dt, L.q8fc2, L.s8fc2, L.rfc2, m.st);
  }
  launch_w8_quantize(m.dt, m.tok_emb, m.d.n_vocab, dt, m.tok8, m.tok8s, nullptr, m.st);
  WMX_HIP(hipStreamSynchronize(m.st));
}

// ------------------------------------------------------------------------------------------------
// context
// ------------------------------------------------------------------------------------------------
struct WindowOut {
  std::vector<int32_t> tokens;
  std::vector<float> jump_times, probs;
};
struct ResultHolder {
  wmx_result r{};
  std::vector<wmx_window_result> win;
  std::vector<WindowOut> data;
};

// in-situ probe launch ids (one decoder layer of a decode step)
// (the six packed projections and the cross attention carry their algorithmic bytes; the others are probed so that
// every launch of the layer's chain has an end time: a launch's in-situ duration is its end minus its predecessor's
// end -- dispatch + execution, the span rocprofv3 reports -- kProbePrev = the previous layer's last launch)
enum {
  kProbeQKV = 0, kProbeOut, kProbeCrossQ, kProbeCrossOut, kProbeFc1, kProbeFc2, kProbeCross, kProbeSelf,
  kProbeRedOut, kProbeRedCrossOut, kProbeRedFc2, kProbePrev, kProbeLaunches = 12
};

// Context groups that decode concurrently on one GPU (wmx_ctx_set_lockstep): a host barrier right before the
// decode loop so that the groups' step graphs start together. In step, the groups run the same launch of the same
// layer at the same time and read its weights once between them (the second reader hits the caches); started a few
// layers apart, each streams the weights from HBM on its own and the decode runs ~5 % slower, a state that persists
// for the whole call because both groups keep the same period (the slow decode mode).
// The same group also meets before every later chunk of 8 decode steps (each member after its previous chunk
// completed), so a perturbation inside a call (a host thread descheduled at a chunk boundary) cannot leave the groups
// apart for the rest of it; that barrier waits only for the members still decoding: a member whose decode loop ends
// (EOT everywhere, or max_new_tokens) leaves it and releases the others.
struct Lockstep {
  std::mutex mu;
  std::condition_variable cv;
  int n = 0, arrived = 0;  // the start barrier: all n members
  unsigned long long gen = 0;
  int active = 0, c_arrived = 0;  // the chunk barrier: the members of the current call still decoding
  unsigned long long c_gen = 0;
  // true when all n members arrived within the timeout (a member that is not decoding costs the others one timeout)
  bool arrive(std::chrono::microseconds timeout) {
    std::unique_lock<std::mutex> lk(mu);
    const unsigned long long g = gen;
    if (++arrived >= n) {
      arrived = 0;
      ++gen;
      active = n;  // every member is in this call's decode loop: a fresh chunk barrier
      c_arrived = 0;
      ++c_gen;
      cv.notify_all();
      return true;
    }
    const bool ok = cv.wait_for(lk, timeout, [&] { return gen != g; });
    if (!ok) --arrived;
    return ok;
  }
  // before a later chunk: true when every member still decoding arrived within the timeout
  bool chunk(std::chrono::microseconds timeout) {
    std::unique_lock<std::mutex> lk(mu);
    const unsigned long long g = c_gen;
    if (++c_arrived >= active) {
      c_arrived = 0;
      ++c_gen;
      cv.notify_all();
      return true;
    }
    const bool ok = cv.wait_for(lk, timeout, [&] { return c_gen != g; });
    if (!ok) --c_arrived;
    return ok;
  }
  // this member's decode loop ended: the others' chunk barriers no longer wait for it
  void leave() {
    std::lock_guard<std::mutex> lk(mu);
    if (active > 0) --active;
    if (c_arrived > 0 && c_arrived >= active) {
      c_arrived = 0;
      ++c_gen;
      cv.notify_all();
    }
  }
};
static std::mutex g_lockstep_mu;
static std::map<int, std::shared_ptr<Lockstep>> g_lockstep;  // by wmx_ctx_set_lockstep key

struct Ctx {
  Model* m = nullptr;
  wmx_opts o{};
  std::vector<int32_t> suppress, align_heads;  // owned copies
  hipStream_t st = nullptr;
  DT dt = DT::BF16;
  int maxB = 1, K = 1, R = 1, Tctx = 448;
  // K = rows per window: beam_size for deterministic search, best_of when sampling (temperature > 0; rows are then
  // independent hypotheses: no beam reorder, no ancestry)
  bool sampling = false, beam = false;
  long max_samples = 480000;
  int fcap = 3001;
  Special sp{51865};
  // ---- buffers ----
  char* buf = nullptr;
  float* pcm = nullptr;
  long* lens = nullptr;
  int* seek = nullptr;
  float *mel_stats = nullptr, *mel = nullptr;  // log-mel block statistics [B][nblk][1 + M], the encoder input
  std::vector<std::pair<size_t, size_t>> guards;  // debug guard gaps (WMX_GUARD), Planner::guards
  long mel_stats_cap = 0;
  uint16_t *im1 = nullptr, *h1 = nullptr, *im2 = nullptr, *ehb = nullptr, *eqkv = nullptr, *eao = nullptr, *ef1 = nullptr,
           *enc_out = nullptr, *ckv = nullptr;
  // fp8 decode: the cross K / V^T images in e4m3 (launch_crosskv_quant of ckv) + one scale per image [L*2][maxB][H]
  uint8_t* ckv8 = nullptr;
  float* ckv8s = nullptr;
  // MX-fp8 encoder operands: e4m3 [rows][K] + e8m0 scales [rows][K/32] (LN out, attention out, fc1 out)
  uint8_t *eh8 = nullptr, *eh8s = nullptr, *ea8 = nullptr, *ea8s = nullptr, *ef8 = nullptr, *ef8s = nullptr;
  float* ex = nullptr;
  // decoder
  int dec_rows_max = 0;  // rows*Tn capacity of the decoder activation buffers
  float* dx = nullptr;
  uint16_t *dhb = nullptr, *dq = nullptr, *dao = nullptr, *dcq = nullptr, *df1 = nullptr, *kc = nullptr, *vc = nullptr;
  float* logits = nullptr;
  int logits_rows = 0;
  int ldl = 0;  // logits row stride (vocab rounded up to 4 floats: 16-B aligned rows)
  float* ws = nullptr;
  long ws_elems = 0;
  float* part = nullptr;  // split-K partials of the packed decode GEMMs [S][rows][N]
  float2* est = nullptr;    // encoder fold: per-256-column (mean, M2) of the residual rows [da / 256][maxB * 1500]
  float2* rstat = nullptr;  // LayerNorm-folded step: per-16-column (mean, M2) of the residual rows [R][dt / 16]
  long part_elems = 0;
  int *hist = nullptr, *hist_tmp = nullptr, *anc = nullptr, *anc_tmp = nullptr, *pad_row = nullptr, *pad_win = nullptr;
  int *slot = nullptr, *n_done = nullptr, *lang_slot = nullptr, *lang_tok = nullptr, *row_map = nullptr, *gather = nullptr;
  float *lang_prob = nullptr, *nospeech = nullptr;
  RowPtrs rp{}, rtmp{};
  BeamState bs{};
  int max_cand = 1;
  int *ctok = nullptr;
  float* clp = nullptr;
  float* sel_ws = nullptr;
  float* xa_ws = nullptr;
  int* xa_cnt = nullptr;
  int* nf_err = nullptr;   // non-finite decode guard (RuleOpts::err): 0, or 1 + row + 1024 * slot of the first hit
  uint32_t* mask = nullptr;
  // alignment
  float *scores = nullptr, *align_out = nullptr, *tprob = nullptr;
  int *a_ntok = nullptr, *a_nframes = nullptr, *a_target = nullptr, *a_heads = nullptr;
  int a_heads_cap = 0;
  // the alignment heads grouped by layer, uploaded once at context creation: layer l's heads are
  // a_heads[a_head_off[l] .. + a_head_cnt[l]) (no per-layer upload and stream sync in the alignment forward)
  std::vector<int> a_head_off, a_head_cnt, a_head_flat;
  // pinned host images of the alignment matrix [B][T][1500] and the text-token probabilities [B][T]: their D2H is a
  // DMA instead of a staged copy into fresh pageable vectors (round 4: 1.4 ms of idle GPU per call and group)
  float *h_align = nullptr, *h_tp = nullptr;
  int* pinned_i = nullptr;
  // decode-step graphs, kept across calls: [0] one step, [1] kGraphChunk steps; valid while graph_key matches
  // (batch, the rule options baked into the captured launches, the probe placement)
  hipGraphExec_t graph[2] = {nullptr, nullptr};
  std::vector<long> graph_key;
  // profiling
  hipEvent_t ev[8];
  // pre-ASR DSP scratch (grown on demand, outside graphs)
  double* dsp_scratch = nullptr;
  size_t dsp_scratch_elems = 0;
  float* dsp_io = nullptr;  // staging of host inputs / outputs
  size_t dsp_io_elems = 0;
  long* dsp_lens = nullptr;
  int dsp_lens_cap = 0;
  // in-situ probe (wmx_ctx_set_probe): [launch][slot][start, end] wall-clock ticks of the probed launches of one
  // decoder layer (kProbe* ids); cur_probe = the buffer of the packed-GEMM launch being issued, or null
  int probe_kernel = -1, probe_layer = 0;
  unsigned long long* probe_buf = nullptr;
  unsigned long long* cur_probe = nullptr;

  double probe_bytes[kProbeLaunches] = {0}, wall_khz = 0;
  int probe_slots[2] = {0, 0};  // [first, last) decode slot probed by the last transcribe
  std::shared_ptr<struct Lockstep> lockstep;  // wmx_ctx_set_lockstep: the decode loops of the group start together
  bool lockstep_ok = false;                   // the last call's barrier saw every member
  long lockstep_timeouts = 0;                 // chunk barriers that timed out (this member then left the barrier)
  bool xq_fused = true;         // decode step: cross-q projection inside the cross attention (WMX_XQ_FUSED=0: off)
  float stage_ms[7] = {0};
  int last_steps = 0;
  // parity recorder (wmx_ctx_record): [cap][R][V] raw logits + [cap][R][2] selections of the last transcribe
  float* rec_logits = nullptr;
  int* rec_sel = nullptr;
  int* rec_base = nullptr;
  int rec_cap = 0, rec_R = 0;
  // word-alignment matrices of the last transcribe (wmx_ctx_alignment_matrix, tests): [B][Tn][1500] as the DTW read
  // them, and per window the text-token count and the content frames
  bool last_align_ok = false;  // h_align holds the last transcribe's matrices
  std::vector<int> last_ntext, last_nframes;
  int last_align_Tn = 0;
};

static void sync_at(Ctx& c, int line) {
  const hipError_t e = hipStreamSynchronize(c.st);
  if (e != hipSuccess)
    throw Error(2, std::string("hipStreamSynchronize(c.st) at wmx_runtime.hip:") + std::to_string(line) + ": " +
                       hipGetErrorString(e));
}
#define sync(c) sync_at(c, __LINE__)


static void alloc_ctx(Ctx& c) {
  const wmx_dims& d = c.m->d;
  const int da = d.n_audio_state, dt = d.n_text_state, M = d.n_mels, V = d.n_vocab, Lt = d.n_text_layer;
  const int B = c.maxB, R = c.R, T = c.Tctx;
  c.fcap = (int)(c.max_samples / 160) + 1;
  c.dec_rows_max = std::max(R, B * T);
  c.logits_rows = std::max({R, 2 * B, 256});
  c.ldl = (V + 3) / 4 * 4;
  int nheads = c.align_heads.empty() ? (Lt - Lt / 2) * d.n_text_head : (int)c.align_heads.size() / 2;
  int heads_per_layer = d.n_text_head;
  c.a_heads_cap = std::max(nheads, heads_per_layer);
  // split-K workspace: up to 8 splits of the widest decoder GEMM (4*dt) over R rows
  c.ws_elems = (long)8 * std::max(R, 64) * 4 * dt;
  Planner P;
  P.guard = getenv("WMX_GUARD") ? 65536 : 0;
  P.add(&c.pcm, (size_t)B * c.max_samples);
  P.add(&c.lens, B);
  P.add(&c.seek, B);
  c.mel_stats_cap = (long)B * logmel_blocks(c.fcap) * (1 + M);
  P.add(&c.mel_stats, (size_t)c.mel_stats_cap);
  P.add(&c.mel, (size_t)B * M * 3000);
  P.add(&c.im1, (size_t)B * 3000 * c.m->K1p);
  P.add(&c.h1, (size_t)B * 3000 * da);
  P.add(&c.im2, (size_t)B * 1500 * 3 * da);
  P.add(&c.ex, (size_t)B * 1500 * da);
  P.add(&c.ehb, (size_t)B * 1500 * da);
  P.add(&c.eqkv, (size_t)B * 1500 * 3 * da);
  P.add(&c.eao, (size_t)B * 1500 * da);
  P.add(&c.ef1, (size_t)B * 1500 * 4 * da);
  P.add(&c.enc_out, (size_t)B * 1500 * da);
  if (c.m->enc_fold) P.add(&c.est, (size_t)(da / 256) * B * 1500);
  if (c.m->mx8) {
    P.add(&c.eh8, (size_t)B * 1500 * da);
    P.add(&c.eh8s, (size_t)B * 1500 * da / 32);
    P.add(&c.ea8, (size_t)B * 1500 * da);
    P.add(&c.ea8s, (size_t)B * 1500 * da / 32);
    P.add(&c.ef8, (size_t)B * 1500 * 4 * da);
    P.add(&c.ef8s, (size_t)B * 1500 * 4 * da / 32);
  }
  P.add(&c.ckv, (size_t)B * kXS * Lt * 2 * dt);  // K and V^T images, key stride kXS (pad stays zero)
  if (c.m->kv8) {
    P.add(&c.ckv8, (size_t)B * kXS * Lt * 2 * dt);
    P.add(&c.ckv8s, (size_t)Lt * 2 * B * d.n_text_head);
  }
  const int DR = c.dec_rows_max;
  P.add(&c.dx, (size_t)DR * dt);
  P.add(&c.dhb, (size_t)DR * dt);
  P.add(&c.dq, (size_t)DR * dt);
  P.add(&c.dao, (size_t)DR * dt);
  P.add(&c.dcq, (size_t)DR * dt);
  P.add(&c.df1, (size_t)DR * 4 * dt);
  P.add(&c.kc, (size_t)Lt * T * R * dt);
  P.add(&c.vc, (size_t)Lt * T * R * dt);
  P.add(&c.logits, (size_t)c.logits_rows * c.ldl);
  P.add(&c.ws, (size_t)c.ws_elems);
  P.add(&c.rstat, (size_t)(dt / 16) * R);
  c.part_elems = (long)R * dt * 48;
  P.add(&c.part, (size_t)c.part_elems);
  P.add(&c.hist, (size_t)R * T);
  P.add(&c.hist_tmp, (size_t)R * T);
  P.add(&c.anc, (size_t)R * T);
  P.add(&c.anc_tmp, (size_t)R * T);
  P.add(&c.pad_row, R);
  P.add(&c.pad_win, B);
  P.add(&c.slot, 4);
  P.add(&c.n_done, 4);
  P.add(&c.lang_slot, B);
  P.add(&c.lang_tok, B);
  P.add(&c.row_map, R);
  P.add(&c.gather, 2 * B + R + B * T);
  P.add(&c.lang_prob, B);
  P.add(&c.nospeech, B);
  for (RowPtrs* rp : {&c.rp, &c.rtmp}) {
    P.add(&rp->ns, R);
    P.add(&rp->last, R);
    P.add(&rp->pen, R);
    P.add(&rp->last_ts, R);
    P.add(&rp->done, R);
    P.add(&rp->sum_lp, R);
  }
  c.max_cand = std::max(1, (int)std::lround(c.K * (double)c.o.patience));
  const int nf = B * c.max_cand;
  P.add(&c.bs.win_done, B);
  P.add(&c.bs.win_active, B);
  P.add(&c.bs.fin_count, B);
  P.add(&c.bs.fin_score, nf);
  P.add(&c.bs.fin_parent, nf);
  P.add(&c.bs.fin_len, nf);
  P.add(&c.bs.fin_hist, (size_t)nf * T);
  P.add(&c.bs.new_parent, R);
  P.add(&c.bs.new_tok, R);
  P.add(&c.bs.new_score, R);
  P.add(&c.ctok, (size_t)R * 9);
  P.add(&c.clp, (size_t)R * 9);
  P.add(&c.sel_ws, logits_select_ws_floats(R, 9));
  // key-chunk records: chunked launches have <= 16 queries per window (more use one chunk, no records)
  P.add(&c.xa_ws, cross_attn_ws_floats(d.n_text_head, B, 16));
  P.add(&c.xa_cnt, (size_t)B * d.n_text_head);
  P.add(&c.nf_err, 4);
  P.add(&c.probe_buf, (size_t)kProbeLaunches * T * kProbeWG * 2);
  P.add(&c.mask, (V + 31) / 32);
  P.add(&c.scores, (size_t)heads_per_layer * B * T * 1500);
  P.add(&c.align_out, (size_t)B * T * 1500);
  P.add(&c.tprob, (size_t)B * T);
  P.add(&c.a_ntok, B);
  P.add(&c.a_nframes, B);
  P.add(&c.a_target, (size_t)B * T);
  P.add(&c.a_heads, c.a_heads_cap + 8);
  WMX_HIP(hipMalloc(&c.buf, P.off));
  WMX_HIP(hipMemsetAsync(c.buf, 0, P.off, c.st));
  for (const auto& g : P.guards) WMX_HIP(hipMemsetAsync(c.buf + g.first, 0xA5, g.second, c.st));
  c.guards = P.guards;
  P.bind(c.buf);
  WMX_HIP(hipHostMalloc(&c.pinned_i, 64));
  // (the pinned alignment images, maxB * 448 * 1500 * 4 bytes, are allocated on the first word-alignment pass: a
  // context without word timestamps never holds them)
  c.a_head_off.assign(Lt, 0);
  c.a_head_cnt.assign(Lt, 0);
  c.a_head_flat.clear();
  for (int l = 0; l < Lt; ++l) {
    c.a_head_off[l] = (int)c.a_head_flat.size();
    for (size_t i = 0; i + 1 < c.align_heads.size(); i += 2)
      if (c.align_heads[i] == l) c.a_head_flat.push_back(c.align_heads[i + 1]);
    c.a_head_cnt[l] = (int)c.a_head_flat.size() - c.a_head_off[l];
  }
  WMX_CHECK((int)c.a_head_flat.size() <= c.a_heads_cap, "alignment heads: table overflow");
  if (!c.a_head_flat.empty())
    WMX_HIP(hipMemcpyAsync(c.a_heads, c.a_head_flat.data(), c.a_head_flat.size() * 4, hipMemcpyHostToDevice, c.st));
  // suppress bitmask
  std::vector<uint32_t> mask((V + 31) / 32, 0u);
  for (int t : c.suppress)
    if (t >= 0 && t < V) mask[t >> 5] |= 1u << (t & 31);
  WMX_HIP(hipMemcpyAsync(c.mask, mask.data(), mask.size() * 4, hipMemcpyHostToDevice, c.st));
  debug_device("ctx alloc");
  for (auto& e : c.ev) WMX_HIP(hipEventCreate(&e));
  {
    int khz = 0;
    WMX_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c.m->device));
    c.wall_khz = khz;
  }
  sync(c);
}

// ------------------------------------------------------------------------------------------------
// GEMM dispatch
// ------------------------------------------------------------------------------------------------
static void gemm(Ctx& c, const uint16_t* A, long lda, const uint16_t* W, long ldw, int M, int N, int K, const Epi& e) {
  GemmCall g;
  g.A = A;
  g.lda = lda;
  g.W = W;
  g.ldw = ldw;
  g.M = M;
  g.N = N;
  g.K = K;
  g.epi = e;
  int bm, bn;
  if (M <= 256 && K % 32 == 0 && N >= 1024) {
    g.tile = TILE_SKINNY;
    launch_gemm(c.dt, g, c.st);
    return;
  }
  if (M >= 4096 && K % WMX_G256_BK == 0 && lda % 8 == 0 && ldw % 8 == 0 && g256_offsets_fit(M, N, lda, ldw) &&
      (e.kind != EPI_CROSSKV || e.d % 256 == 0) && e.kind != EPI_QKV_CACHE) {
    // encoder / conv front end / cross-K/V: 256x256 ping-pong tile, every tile on its own CU
    g.tile = TILE_256;
    launch_gemm(c.dt, g, c.st);
    return;
  }
  // rows from which the 128x128 tile is used (the word-alignment forward, ~900 rows per context group: align stage
  // 15.7-16.3 vs 16.9-18.8 ms with 64x64 tiles, profiles/r03r_align_m128_ab.txt)
  if (M >= 512) {
    g.tile = TILE_128x128;
    bm = 128;
    bn = 128;
  } else if (M > 32) {
    g.tile = TILE_64x64;
    bm = 64;
    bn = 64;
  } else {
    g.tile = TILE_32x64;
    bm = 32;
    bn = 64;
  }
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  int splits = 1;
  if (tiles < 200 && K >= 512) {
    splits = (int)std::min<long>({8, K / 256, (256 + tiles - 1) / tiles});
    while (splits > 1 && (long)splits * M * N > c.ws_elems) --splits;
  }
  g.splits = splits;
  g.ws = c.ws;
  g.ws_elems = c.ws_elems;
  launch_gemm(c.dt, g, c.st);
}

static Epi epi(int kind, const float* bias, void* out, long ldc) {
  Epi e;
  e.kind = kind;
  e.bias = bias;
  e.out = out;
  e.ldc = ldc;
  return e;
}

// decoder projection: packed weights (decode, few rows), or the row-major copy on the tiled MFMA GEMM when there
// are many rows (prompt prefill, word alignment: the packed kernel would re-read the weights per 64-row chunk)
// An 8-bit weight (fp8 decode): q8 (packed8_index) + per-row scales s8; the packed kernel then reads q8 instead of Wp.
struct W8 {
  const uint8_t* q8 = nullptr;
  const float* s8 = nullptr;
  bool i8 = false;  // int8 bytes (the CTranslate2 grid) instead of e4m3
};
static void set_w(PackedCall& g, const uint16_t* Wp, W8 w8) {
  g.W = w8.q8 ? reinterpret_cast<const uint16_t*>(w8.q8) : Wp;
  g.wscale = w8.q8 ? w8.s8 : nullptr;
  g.w8kind = w8.i8 ? 2 : 1;
}

static void gemm_p(Ctx& c, const uint16_t* A, long lda, const uint16_t* Wp, int M, int N, int K, const Epi& e,
                   const uint16_t* Wrm = nullptr, W8 w8 = {}) {
  if (Wrm && M > 256) {  // (fp8 decode: Wrm holds the dequantized 8-bit weights)
    gemm(c, A, lda, Wrm, K, M, N, K, e);
    return;
  }
  PackedCall g;
  g.A = A;
  g.lda = lda;
  set_w(g, Wp, w8);
  g.M = M;
  g.N = N;
  g.K = K;
  g.S = 1;
  g.epi = e;
  g.tprobe = c.cur_probe;
  g.pslot = c.slot;
  launch_gemm_packed(c.dt, g, c.st);
}

// decoder projection on packed weights, split-K raw partials into c.part; returns the split count
static int gemm_p_part(Ctx& c, const uint16_t* A, long lda, const uint16_t* Wp, int M, int N, int K, W8 w8 = {}) {
  PackedCall g;
  g.A = A;
  g.lda = lda;
  set_w(g, Wp, w8);
  g.M = M;
  g.N = N;
  g.K = K;
  g.S = packed_splits(M, N, K, c.part_elems);
  g.part = c.part;
  g.tprobe = c.cur_probe;
  g.pslot = c.slot;
  if (g.S == 1) {  // nothing to split: a single slice is still written as raw partials
    g.S = 2;
    WMX_CHECK(2L * M * N <= c.part_elems, "decode gemm: partial buffer too small");
  }
  launch_gemm_packed(c.dt, g, c.st);
  return g.S;
}

// decoder projection whose split-K partials feed x += bias + sum; out16 = LN(x): the GEMM, then reduce_ln
// (an in-launch reduce + LayerNorm tail measured slower than the kernel boundary, 798 vs 587 ms per call, and was
// removed in round 6)
static void gemm_p_redln(Ctx& c, const uint16_t* A, long lda, const uint16_t* Wp, int M, int N, int K,
                         const float* bias, const float* g, const float* b, unsigned long long* redprobe = nullptr,
                         W8 w8 = {}) {
  const int S = gemm_p_part(c, A, lda, Wp, M, N, K, w8);
  c.cur_probe = nullptr;
  launch_reduce_ln(c.dt, c.part, S, bias, c.dx, g, b, c.dhb, M, N, c.st, redprobe, c.slot);
}

// ------------------------------------------------------------------------------------------------
// encoder
// ------------------------------------------------------------------------------------------------
// MX-fp8 encoder layers (BASELINE config 5): the four projections of every layer run on
// v_mfma_scale_f32_16x16x128_f8f6f4 with their A operands produced directly in MX-fp8 by the LayerNorm, the
// attention epilogue and the fc1 GELU epilogue; q/k/v, the attention itself and the fp32 residual stay as in
// the 16-bit path.
static void gemm_mx8(Ctx& c, const uint8_t* A, const uint8_t* AS, const uint8_t* W, const uint8_t* WS, int M, int N,
                     int K, const Epi& e) {
  Mx8Call g;
  g.A = A;
  g.lda = K;
  g.AS = AS;
  g.ldas = K / 32;
  g.W = W;
  g.ldw = K;
  g.WS = WS;
  g.ldws = K / 32;
  g.M = M;
  g.N = N;
  g.K = K;
  g.epi = e;
  launch_gemm_mx8(c.dt, g, c.st);
}

static void encode_layers_mx8(Ctx& c, int B) {
  Model& m = *c.m;
  const int da = m.d.n_audio_state, H = m.d.n_audio_head;
  const int rows = B * 1500;
  for (auto& L : m.enc) {
    launch_layernorm_mx8(c.ex, L.ln1g, L.ln1b, c.eh8, c.eh8s, rows, da, c.st);
    Epi eq;
    eq.kind = EPI_STORE16;
    eq.bias = L.bqkv;
    eq.out = c.eqkv;
    eq.ldc = 3L * da;
    gemm_mx8(c, c.eh8, c.eh8s, L.qkv8, L.qkv8s, rows, 3 * da, da, eq);
    AttnArgs a{};
    a.q = c.eqkv;
    a.k = c.eqkv + da;
    a.v = c.eqkv + 2 * da;
    a.q_ld = a.k_ld = a.v_ld = 3 * da;
    a.q_bstride = a.k_bstride = a.v_bstride = 1500L * 3 * da;
    a.o = c.eao;
    a.o_ld = da;
    a.o_bstride = 1500L * da;
    a.B = B;
    a.H = H;
    a.Tq = a.Tk = 1500;
    a.head_stride = 64;
    a.o8 = c.ea8;
    a.os = c.ea8s;
    a.o8_ld = da;
    a.os_ld = da / 32;
    launch_attn_encoder(c.dt, a, c.st);
    Epi eo;
    eo.kind = EPI_RESID32;
    eo.bias = L.bo;
    eo.out = c.ex;
    eo.ldc = da;
    gemm_mx8(c, c.ea8, c.ea8s, L.o8, L.o8s, rows, da, da, eo);
    launch_layernorm_mx8(c.ex, L.ln2g, L.ln2b, c.eh8, c.eh8s, rows, da, c.st);
    Epi e1;
    e1.kind = EPI_GELU_MX8;
    e1.bias = L.bfc1;
    e1.out = c.ef8;
    e1.ldc = 4L * da;
    e1.out2 = c.ef8s;
    e1.ldc2 = 4L * da / 32;
    gemm_mx8(c, c.eh8, c.eh8s, L.fc18, L.fc18s, rows, 4 * da, da, e1);
    Epi e2;
    e2.kind = EPI_RESID32;
    e2.bias = L.bfc2;
    e2.out = c.ex;
    e2.ldc = da;
    gemm_mx8(c, c.ef8, c.ef8s, L.fc28, L.fc28s, rows, da, 4 * da, e2);
  }
}

// encoder pass on the 256 x 256 GEMM with the LayerNorms folded (Model::enc_fold): the residual stream is two 16-bit
// planes x = hi + lo (hi in ehb, lo in ex's storage; ~17 significant bits, the fp32 row's bytes), which the residual
// producers (conv2, out-proj, fc2) update together with the row statistics per 256 columns (est); qkv and fc1
// multiply hi by W diag(g) and finish LN in their epilogue, rstd (acc - mean c1) + c2 (wmx_gemm.hip).  No LayerNorm
// launches inside the stack; the final one (ln_post) reads the planes.  Numerics: x enters the projections rounded
// to 16 bits before the mean is removed, which adds ~2^-9 |mean| / std relative error per projection input on top of
// the unfolded form's LN-output rounding ("Encoder LayerNorm fold").
static bool enc_fold_rows(const Ctx& c, long rows) {
  // the gemm256 dispatch condition of gemm() for every folded launch (the widest A: fc2's 4 d columns)
  const long da = c.m->d.n_audio_state;
  return c.m->enc_fold && c.est && rows >= 4096 && g256_offsets_fit(rows, 4 * da, 4 * da, 4 * da);
}

static Epi epi_lns(Ctx& c, int kind, const float* bias, long rows) {
  Epi e = epi(kind, bias, c.ex, c.m->d.n_audio_state);
  e.out16 = c.ehb;
  e.stats = c.est;
  e.stats_ld = rows;
  return e;
}

static Epi epi_lnf(Ctx& c, int kind, const float* c1, const float* c2, void* out, long ldc, long rows) {
  Epi e = epi(kind, c2, out, ldc);
  e.c1 = c1;
  e.stats = c.est;
  e.stats_ld = rows;
  e.lng = c.m->d.n_audio_state / 256;
  return e;
}

static void encode(Ctx& c, int B) {
  Model& m = *c.m;
  const int da = m.d.n_audio_state, H = m.d.n_audio_head, M = m.d.n_mels;
  const long rows = (long)B * 1500;
  const bool fold = !m.mx8 && enc_fold_rows(c, rows);
  launch_im2col_conv1(c.dt, c.mel, B, M, m.K1p, c.im1, c.st);
  gemm(c, c.im1, m.K1p, m.conv1w, m.K1p, B * 3000, da, m.K1p, epi(EPI_GELU16, m.conv1b, c.h1, da));
  launch_im2col_conv2(c.dt, c.h1, B, da, c.im2, c.st);
  Epi e2 = fold ? epi_lns(c, EPI_GELU_POS32_LNS, m.conv2b, rows) : epi(EPI_GELU_POS32, m.conv2b, c.ex, da);
  e2.pos = m.enc_pos;
  e2.posT = 1500;
  gemm(c, c.im2, 3 * da, m.conv2w, 3 * da, (int)rows, da, 3 * da, e2);
  if (m.mx8) {
    encode_layers_mx8(c, B);
    launch_layernorm(c.dt, c.ex, m.lnpg, m.lnpb, c.enc_out, (int)rows, da, c.st);
    return;
  }
  for (size_t l = 0; l < m.enc.size(); ++l) {
    const EncLayer& L = m.enc[l];
    if (fold) {
      gemm(c, c.ehb, da, L.fqkv, da, (int)rows, 3 * da, da,
           epi_lnf(c, EPI_LNF_STORE16, L.c1qkv, L.c2qkv, c.eqkv, 3 * da, rows));
    } else {
      launch_layernorm(c.dt, c.ex, L.ln1g, L.ln1b, c.ehb, (int)rows, da, c.st);
      gemm(c, c.ehb, da, L.wqkv, da, (int)rows, 3 * da, da, epi(EPI_STORE16, L.bqkv, c.eqkv, 3 * da));
    }
    AttnArgs a{};
    a.q = c.eqkv;
    a.k = c.eqkv + da;
    a.v = c.eqkv + 2 * da;
    a.q_ld = a.k_ld = a.v_ld = 3 * da;
    a.q_bstride = a.k_bstride = a.v_bstride = 1500L * 3 * da;
    a.o = c.eao;
    a.o_ld = da;
    a.o_bstride = 1500L * da;
    a.B = B;
    a.H = H;
    a.Tq = a.Tk = 1500;
    a.head_stride = 64;
    launch_attn_encoder(c.dt, a, c.st);
    if (fold) {
      gemm(c, c.eao, da, L.wo, da, (int)rows, da, da, epi_lns(c, EPI_RESID32_LNS, L.bo, rows));
      gemm(c, c.ehb, da, L.ffc1, da, (int)rows, 4 * da, da,
           epi_lnf(c, EPI_LNF_GELU16, L.c1fc1, L.c2fc1, c.ef1, 4 * da, rows));
      gemm(c, c.ef1, 4 * da, L.wfc2, 4 * da, (int)rows, da, 4 * da, epi_lns(c, EPI_RESID32_LNS, L.bfc2, rows));
    } else {
      gemm(c, c.eao, da, L.wo, da, (int)rows, da, da, epi(EPI_RESID32, L.bo, c.ex, da));
      launch_layernorm(c.dt, c.ex, L.ln2g, L.ln2b, c.ehb, (int)rows, da, c.st);
      gemm(c, c.ehb, da, L.wfc1, da, (int)rows, 4 * da, da, epi(EPI_GELU16, L.bfc1, c.ef1, 4 * da));
      gemm(c, c.ef1, 4 * da, L.wfc2, 4 * da, (int)rows, da, 4 * da, epi(EPI_RESID32, L.bfc2, c.ex, da));
    }
  }
  if (fold)
    launch_layernorm_split(c.dt, c.ehb, reinterpret_cast<const uint16_t*>(c.ex), m.lnpg, m.lnpb, c.enc_out, (int)rows,
                           da, c.st);
  else
    launch_layernorm(c.dt, c.ex, m.lnpg, m.lnpb, c.enc_out, (int)rows, da, c.st);
}

// layer l's cross K / V in the head-major layout written by EPI_CROSSKV
static const uint16_t* cross_k(const Ctx& c, int l) {
  return c.ckv + (size_t)(2 * l) * c.maxB * kXS * c.m->d.n_text_state;
}
static const uint16_t* cross_v(const Ctx& c, int l) {
  return c.ckv + (size_t)(2 * l + 1) * c.maxB * kXS * c.m->d.n_text_state;
}

// the cross-attention images of layer l on a decoder-attention call: the 16-bit images, or (fp8 decode) the e4m3
// images and their per-(window, head) scales
static void set_cross_images(const Ctx& c, DecAttnArgs& a, int l) {
  const Model& m = *c.m;
  a.x_wstride = (long)kXS * m.d.n_text_state;
  a.x_hstride = (long)kXS * 64;
  if (m.kv8) {
    const size_t img = (size_t)c.maxB * kXS * m.d.n_text_state;  // bytes per (layer, kv) block of images
    const size_t nsc = (size_t)c.maxB * m.d.n_text_head;
    a.ck = reinterpret_cast<const uint16_t*>(c.ckv8 + (2 * l) * img);
    a.cv = reinterpret_cast<const uint16_t*>(c.ckv8 + (2 * l + 1) * img);
    a.ck_scale = c.ckv8s + (2 * l) * nsc;
    a.cv_scale = c.ckv8s + (2 * l + 1) * nsc;
  } else {
    a.ck = cross_k(c, l);
    a.cv = cross_v(c, l);
  }
}

// the 8-bit copy of a decoder projection (fp8 decode), or none
static W8 w8_of(const Model& m, const uint8_t* q, const float* s) { return m.w8 ? W8{q, s, m.i8} : W8{}; }

static void cross_kv(Ctx& c, int B) {
  Model& m = *c.m;
  const int dt = m.d.n_text_state, Lt = m.d.n_text_layer;
  WMX_CHECK(m.d.n_audio_state == dt, "cross K/V: audio and text widths differ");
  Epi e = epi(EPI_CROSSKV, m.bckv, c.ckv, 0);
  e.d = dt;
  e.xw = c.maxB;
  e.xt = 1500;
  gemm(c, c.enc_out, dt, m.wckv, dt, B * 1500, Lt * 2 * dt, dt, e);
  // fp8 decode: every (layer-kv, window, head) image to e4m3 with its own power-of-two scale (once per call; the
  // decode steps then stream half the bytes)
  if (m.kv8) launch_crosskv_quant(c.ckv, c.ckv8, c.ckv8s, 2 * Lt, c.maxB, B, m.d.n_text_head, c.st);
}

// ------------------------------------------------------------------------------------------------
// decoder forward
//   rows sequences x Tn new tokens at slots *slot .. *slot+Tn-1.  Token of (r, i) = tok[r*tok_ld + slot + i].
//   The KV cache row of sequence r is r*rmul.  prefill: flash kernels (causal, first valid key pad_seq[r]);
//   decode (Tn == 1): gather kernels through `anc` (null -> identity).  `align`: alignment-head scores.
// ------------------------------------------------------------------------------------------------
struct FwdArgs {
  int rows, Tn, rmul;
  const int* tok;
  long tok_ld;
  const int* pad_seq;  // per sequence (embed positions + flash kbegin)
  bool prefill;
  const int* anc;
  bool align = false;
  int win_rows = 0;  // decode step: rows per window of the cross attention (0: the context's beam width)
};

// Decode step (Tn == 1): every projection runs on packed weights with split-K partials, and the reductions are
// fused into the consumers -- q/k/v into self attention (which also writes the KV cache), cross q into cross
// attention, out-proj / fc2 into reduce_ln (residual add + the next LayerNorm).  10 launches per layer.
// Leaves LN_final(x) of every row in c.dhb.
static void dec_step_fast(Ctx& c, const FwdArgs& f) {
  Model& m = *c.m;
  const int dt = m.d.n_text_state, H = m.d.n_text_head, Lt = m.d.n_text_layer;
  const int R = f.rows;
  const size_t cache_layer = (size_t)c.Tctx * c.R * dt;
  launch_embed_ln(c.dt, m.tok_emb, m.dec_pos, f.tok, f.tok_ld, R, f.pad_seq, c.slot, m.dec[0].ln1g, m.dec[0].ln1b, dt,
                  c.dx, c.dhb, c.st, m.d.n_vocab);
  const size_t probe_stride = (size_t)c.Tctx * kProbeWG * 2;
  for (int l = 0; l < Lt; ++l) {
    DecLayer& L = m.dec[l];
    const bool last = l + 1 == Lt;
    const bool probed = c.probe_kernel >= 0 && l == c.probe_layer;
    const bool prev = c.probe_kernel >= 0 && l + 1 == c.probe_layer;  // its last launch precedes the probed qkv
    auto probe = [&](int id) { c.cur_probe = probed ? c.probe_buf + id * probe_stride : nullptr; };
    auto pbuf = [&](int id) { return probed ? c.probe_buf + id * probe_stride : nullptr; };
    // self attention: QKV partials -> (reduce, cache write, attention) -> out-proj partials -> +x, LN2
    probe(kProbeQKV);
    int S = gemm_p_part(c, c.dhb, dt, L.wqkv, R, 3 * dt, dt, w8_of(m, L.q8qkv, L.s8qkv));
    c.cur_probe = nullptr;
    DecAttnArgs a{};
    a.o = c.dao;
    a.R = R;
    a.Tn = 1;
    a.H = H;
    a.d = dt;
    a.kc = c.kc + l * cache_layer;
    a.vc = c.vc + l * cache_layer;
    a.kv_R = c.R;
    a.anc = f.anc;
    a.anc_ld = c.Tctx;
    a.pad = f.pad_seq;
    a.slot0 = c.slot;
    a.qpart = c.part;
    a.qS = S;
    a.qpart_stride = (long)R * 3 * dt;
    a.qpart_ld = 3 * dt;
    a.qbias = L.bqkv;
    a.tprobe = pbuf(kProbeSelf);
    launch_self_attn(c.dt, a, c.st);
    probe(kProbeOut);
    gemm_p_redln(c, c.dao, dt, L.wo, R, dt, dt, L.bo, L.ln2g, L.ln2b, pbuf(kProbeRedOut), w8_of(m, L.q8o, L.s8o));
    // cross attention: q partials -> (reduce, attention) -> out-proj partials -> +x, LN3; with c.xq_fused the
    // cross attention projects its own queries from LN2(x) (no cross-q launch)
    if (!c.xq_fused) {
      probe(kProbeCrossQ);
      S = gemm_p_part(c, c.dhb, dt, L.wcq, R, dt, dt, w8_of(m, L.q8cq, L.s8cq));
      c.cur_probe = nullptr;
    }
    DecAttnArgs x{};
    x.o = c.dao;
    x.R = R;
    x.Tn = 1;
    x.H = H;
    x.d = dt;
    set_cross_images(c, x, l);
    x.Tk = 1500;
    x.rows_per_win = f.win_rows > 0 ? f.win_rows : c.K;
    x.qpart = c.part;
    x.qS = S;
    x.qpart_stride = (long)R * dt;
    x.qpart_ld = dt;
    x.qbias = L.bcq;
    if (c.xq_fused) {
      x.qS = 0;
      x.wq = m.kv8 ? reinterpret_cast<const uint16_t*>(L.q8cq) : L.wcq;
      x.wq_scale = m.kv8 ? L.s8cq : nullptr;
      x.qin = c.dhb;
      x.qin_ld = dt;
    }
    x.xcnt = c.xa_cnt;
    x.slot0 = c.slot;
    if (probed) x.tprobe = c.probe_buf + kProbeCross * probe_stride;
    launch_cross_attn(c.dt, x, c.xa_ws, c.st);
    probe(kProbeCrossOut);
    gemm_p_redln(c, c.dao, dt, L.wco, R, dt, dt, L.bco, L.ln3g, L.ln3b, pbuf(kProbeRedCrossOut),
                 w8_of(m, L.q8co, L.s8co));
    // MLP: fc1 (+bias, GELU in-kernel) -> fc2 partials -> +x, next LN1 (or the final LN)
    probe(kProbeFc1);
    gemm_p(c, c.dhb, dt, L.wfc1, R, 4 * dt, dt, epi(EPI_GELU16, L.bfc1, c.df1, 4 * dt), nullptr,
           w8_of(m, L.q8fc1, L.s8fc1));
    probe(kProbeFc2);
    gemm_p_redln(c, c.df1, 4 * dt, L.wfc2, R, dt, 4 * dt, L.bfc2, last ? m.lng : m.dec[l + 1].ln1g,
                 last ? m.lnb : m.dec[l + 1].ln1b,
                 probed ? pbuf(kProbeRedFc2) : prev ? c.probe_buf + kProbePrev * probe_stride : nullptr,
                 w8_of(m, L.q8fc2, L.s8fc2));
    c.cur_probe = nullptr;
  }
}

// The mixed step's residual producers: x += acc + bias, its 16-bit copy and per-16-column row statistics
static Epi epi_resid_stats(Ctx& c, const float* bias, int R) {
  Epi e = epi(EPI_RESID_STATS, bias, c.dx, c.m->d.n_text_state);
  e.out16 = c.dhb;
  e.stats = c.rstat;
  e.stats_ld = c.m->d.n_text_state / 16;  // row stride of [R][dt / 16]
  return e;
}

static void gemm_p_resid(Ctx& c, const uint16_t* A, long lda, const uint16_t* Wp, int M, int N, int K, const Epi& e) {
  PackedCall g;
  g.A = A;
  g.lda = lda;
  g.W = Wp;
  g.M = M;
  g.N = N;
  g.K = K;
  g.S = 1;
  g.epi = e;
  g.nct = 1;  // unsplit: 16 columns per workgroup (N / 16 workgroups, 16 waves splitting K)
  g.tprobe = c.cur_probe;
  g.pslot = c.slot;
  launch_gemm_packed(c.dt, g, c.st);
}

// WMX_DEBUG_SYNC=1 (fault localisation on eager, uncaptured steps): synchronise after each launch of the step
// and name the launch that failed
static void debug_sync(Ctx& c, const char* what, int l) {
  static const bool on = getenv("WMX_DEBUG_SYNC") != nullptr;
  if (!on) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  WMX_HIP(hipStreamIsCapturing(c.st, &cs));
  if (cs != hipStreamCaptureStatusNone) return;
  const hipError_t e = hipStreamSynchronize(c.st);
  if (e != hipSuccess) throw std::runtime_error(std::string("debug sync after ") + what + " (layer " + std::to_string(l) + "): " + hipGetErrorString(e));
}


// The mixed decode step: dec_step_fast with the two d x d residual producers of every layer (out-projection,
// cross out-projection) unsplit -- x += acc + bias, its 16-bit copy and per-16-column row statistics in the GEMM
// epilogue (EPI_RESID_STATS) -- so their reduce_ln launches go: LN2 is applied by the fused cross-q projection
// through W diag(g2), c1, c2 (the cross attention merges the row statistics it loads beside its K batch), LN3 by fc1's
// folded GELU epilogue.  fc2 (K = 4d) keeps split-K partials + reduce_ln (its unsplit form is 15 vs 11 us, DESIGN.md
// §3), which also produces the next layer's LN1 rows for the split-K QKV.  8 launches per layer instead of 10.
// Leaves LN_final(x) of every row in c.dhb.
static void dec_step_mixed(Ctx& c, const FwdArgs& f) {
  Model& m = *c.m;
  const int dt = m.d.n_text_state, H = m.d.n_text_head, Lt = m.d.n_text_layer;
  const int R = f.rows;
  const size_t cache_layer = (size_t)c.Tctx * c.R * dt;
  launch_embed_ln(c.dt, m.tok_emb, m.dec_pos, f.tok, f.tok_ld, R, f.pad_seq, c.slot, m.dec[0].ln1g, m.dec[0].ln1b, dt,
                  c.dx, c.dhb, c.st, m.d.n_vocab);
  const size_t probe_stride = (size_t)c.Tctx * kProbeWG * 2;
  for (int l = 0; l < Lt; ++l) {
    DecLayer& L = m.dec[l];
    const bool last = l + 1 == Lt;
    const bool probed = c.probe_kernel >= 0 && l == c.probe_layer;
    const bool prev = c.probe_kernel >= 0 && l + 1 == c.probe_layer;
    auto probe = [&](int id) { c.cur_probe = probed ? c.probe_buf + id * probe_stride : nullptr; };
    auto pbuf = [&](int id) { return probed ? c.probe_buf + id * probe_stride : nullptr; };
    // self attention on LN1(x) (c.dhb): QKV partials -> (reduce, cache write, attention)
    probe(kProbeQKV);
    const int S = gemm_p_part(c, c.dhb, dt, L.wqkv, R, 3 * dt, dt);
    c.cur_probe = nullptr;
    DecAttnArgs a{};
    a.o = c.dao;
    a.R = R;
    a.Tn = 1;
    a.H = H;
    a.d = dt;
    a.kc = c.kc + l * cache_layer;
    a.vc = c.vc + l * cache_layer;
    a.kv_R = c.R;
    a.anc = f.anc;
    a.anc_ld = c.Tctx;
    a.pad = f.pad_seq;
    a.slot0 = c.slot;
    a.qpart = c.part;
    a.qS = S;
    a.qpart_stride = (long)R * 3 * dt;
    a.qpart_ld = 3 * dt;
    a.qbias = L.bqkv;
    a.tprobe = pbuf(kProbeSelf);
    launch_self_attn(c.dt, a, c.st);
    // out-projection, unsplit: x += o Wo^T + bo, x16 -> c.dhb, row statistics -> c.rstat
    probe(kProbeOut);
    gemm_p_resid(c, c.dao, dt, L.wo, R, dt, dt, epi_resid_stats(c, L.bo, R));
    c.cur_probe = nullptr;
    // cross attention with the fused, LN2-folded query projection of x16
    DecAttnArgs x{};
    x.o = c.dao;
    x.R = R;
    x.Tn = 1;
    x.H = H;
    x.d = dt;
    set_cross_images(c, x, l);
    x.Tk = 1500;
    x.rows_per_win = f.win_rows > 0 ? f.win_rows : c.K;
    x.wq = L.fcq;
    x.qin = c.dhb;
    x.qin_ld = dt;
    x.ln_c1 = L.c1cq;
    x.ln_c2 = L.c2cq;
    x.ln_stats = c.rstat;
    x.ln_ld = dt / 16;
    x.xcnt = c.xa_cnt;
    x.slot0 = c.slot;
    if (probed) x.tprobe = c.probe_buf + kProbeCross * probe_stride;
    launch_cross_attn(c.dt, x, c.xa_ws, c.st);
    // cross out-projection, unsplit: x += o Wco^T + bco, x16, statistics
    probe(kProbeCrossOut);
    gemm_p_resid(c, c.dao, dt, L.wco, R, dt, dt, epi_resid_stats(c, L.bco, R));
    // MLP: GELU(LN3-folded fc1 of x16) -> fc2 partials -> reduce_ln (x += ..., next layer's LN1 or the final LN)
    probe(kProbeFc1);
    Epi e1 = epi(EPI_LNFOLD_GELU16, nullptr, c.df1, 4 * dt);
    e1.c1 = L.c1fc1;
    e1.c2 = L.c2fc1;
    e1.stats = c.rstat;
    e1.stats_ld = dt / 16;
    gemm_p(c, c.dhb, dt, L.ffc1, R, 4 * dt, dt, e1);
    probe(kProbeFc2);
    gemm_p_redln(c, c.df1, 4 * dt, L.wfc2, R, dt, 4 * dt, L.bfc2, last ? m.lng : m.dec[l + 1].ln1g,
                 last ? m.lnb : m.dec[l + 1].ln1b,
                 probed ? pbuf(kProbeRedFc2) : prev ? c.probe_buf + kProbePrev * probe_stride : nullptr);
    c.cur_probe = nullptr;
  }
}

static void dec_step(Ctx& c, const FwdArgs& f) {
  if (c.m->mixed && c.xq_fused)
    dec_step_mixed(c, f);
  else
    dec_step_fast(c, f);
}

static void dec_forward(Ctx& c, const FwdArgs& f) {
  Model& m = *c.m;
  const int dt = m.d.n_text_state, H = m.d.n_text_head, Lt = m.d.n_text_layer;
  const int rowsT = f.rows * f.Tn;
  WMX_CHECK(rowsT <= c.dec_rows_max, "decoder: too many rows");
  launch_embed(c.dt, m.tok_emb, m.dec_pos, f.tok, f.tok_ld, f.rows, f.Tn, f.pad_seq, c.slot, dt, c.dx, c.st, m.d.n_vocab);
  const size_t cache_layer = (size_t)c.Tctx * c.R * dt;
  for (int l = 0; l < Lt; ++l) {
    DecLayer& L = m.dec[l];
    uint16_t* kcl = c.kc + l * cache_layer;
    uint16_t* vcl = c.vc + l * cache_layer;
    launch_layernorm(c.dt, c.dx, L.ln1g, L.ln1b, c.dhb, rowsT, dt, c.st);
    Epi eq = epi(EPI_QKV_CACHE, L.bqkv, c.dq, dt);
    eq.d = dt;
    eq.Tn = f.Tn;
    eq.R = c.R;
    eq.rmul = f.rmul;
    eq.slot0 = c.slot;
    eq.kc = kcl;
    eq.vc = vcl;
    gemm_p(c, c.dhb, dt, L.wqkv, rowsT, 3 * dt, dt, eq, L.rqkv, w8_of(m, L.q8qkv, L.s8qkv));
    if (f.prefill) {
      AttnArgs a{};
      a.q = c.dq;
      a.q_ld = dt;
      a.q_bstride = (long)f.Tn * dt;
      a.k = kcl;
      a.v = vcl;
      a.k_ld = a.v_ld = (long)c.R * dt;
      a.k_bstride = a.v_bstride = (long)f.rmul * dt;
      a.o = c.dao;
      a.o_ld = dt;
      a.o_bstride = (long)f.Tn * dt;
      a.B = f.rows;
      a.H = H;
      a.Tq = f.Tn;
      a.Tk = f.Tn;  // prefill always starts at slot 0
      a.head_stride = 64;
      launch_attn_flash(c.dt, a, 1, 0, f.pad_seq, c.st);
    } else {
      DecAttnArgs a{};
      a.q = c.dq;
      a.q_ld = dt;
      a.o = c.dao;
      a.R = f.rows;
      a.Tn = 1;
      a.H = H;
      a.d = dt;
      a.kc = kcl;
      a.vc = vcl;
      a.kv_R = c.R;
      a.anc = f.anc;
      a.anc_ld = c.Tctx;
      a.pad = f.pad_seq;
      a.slot0 = c.slot;
      launch_self_attn(c.dt, a, c.st);
    }
    gemm_p(c, c.dao, dt, L.wo, rowsT, dt, dt, epi(EPI_RESID32, L.bo, c.dx, dt), L.ro, w8_of(m, L.q8o, L.s8o));
    launch_layernorm(c.dt, c.dx, L.ln2g, L.ln2b, c.dhb, rowsT, dt, c.st);
    gemm_p(c, c.dhb, dt, L.wcq, rowsT, dt, dt, epi(EPI_STORE16, L.bcq, c.dcq, dt), L.rcq, w8_of(m, L.q8cq, L.s8cq));
    {
      DecAttnArgs a{};
      a.q = c.dcq;
      a.q_ld = dt;
      a.o = c.dao;
      a.R = f.rows;
      a.Tn = f.Tn;
      a.H = H;
      a.d = dt;
      set_cross_images(c, a, l);
      a.Tk = 1500;
      // prefill: one sequence per window; decode through this path: the beams of a window share it
      a.rows_per_win = f.prefill ? 1 : c.K;
      a.xcnt = c.xa_cnt;
      launch_cross_attn(c.dt, a, c.xa_ws, c.st);
    }
    if (f.align && c.a_head_cnt[l] > 0) {  // this layer's alignment heads (the device table, alloc_ctx)
      const int nh = c.a_head_cnt[l];
      {
        DecAttnArgs a{};
        a.q = c.dcq;
        a.q_ld = dt;
        a.R = f.rows;
        a.Tn = f.Tn;
        a.H = H;
        a.d = dt;
        set_cross_images(c, a, l);
        a.Tk = 1500;
        a.rows_per_win = 1;
        launch_cross_scores(c.dt, a, c.a_heads + c.a_head_off[l], nh, c.scores, c.st);
        launch_align_matrix_acc(c.scores, nh, rowsT, 1500, f.Tn, c.a_ntok, c.a_nframes, c.o.median_filter_width,
                                f.rows, c.st, c.align_out);
      }
    }
    gemm_p(c, c.dao, dt, L.wco, rowsT, dt, dt, epi(EPI_RESID32, L.bco, c.dx, dt), L.rco, w8_of(m, L.q8co, L.s8co));
    launch_layernorm(c.dt, c.dx, L.ln3g, L.ln3b, c.dhb, rowsT, dt, c.st);
    gemm_p(c, c.dhb, dt, L.wfc1, rowsT, 4 * dt, dt, epi(EPI_GELU16, L.bfc1, c.df1, 4 * dt), L.rfc1,
           w8_of(m, L.q8fc1, L.s8fc1));
    gemm_p(c, c.df1, 4 * dt, L.wfc2, rowsT, dt, 4 * dt, epi(EPI_RESID32, L.bfc2, c.dx, dt), L.rfc2,
           w8_of(m, L.q8fc2, L.s8fc2));
  }
}

// final LN of selected rows + logits GEMM into c.logits [n][V]
// (ln_done: c.dhb already holds LN_final of rows 0..n-1, as dec_step_fast leaves it)
static void dec_logits(Ctx& c, const int* rows_idx, int n, bool ln_done = false) {
  Model& m = *c.m;
  const int dt = m.d.n_text_state, V = m.d.n_vocab;
  WMX_CHECK(n <= c.logits_rows, "logits: too many rows");
  if (!ln_done) launch_layernorm_rows(c.dt, c.dx, rows_idx, m.lng, m.lnb, c.dhb, n, dt, c.st);
  gemm_p(c, c.dhb, dt, m.tok_emb, n, V, dt, epi(EPI_STORE32, nullptr, c.logits, c.ldl), nullptr,
         w8_of(m, m.tok8, m.tok8s));
}

static void set_slot(Ctx& c, int v) {
  c.pinned_i[0] = v;
  WMX_HIP(hipMemcpyAsync(c.slot, c.pinned_i, 4, hipMemcpyHostToDevice, c.st));
  sync(c);
}

// ------------------------------------------------------------------------------------------------
// DTW (openai timing.dtw_cpu + backtrace), float32 cost accumulation like the oracle
// ------------------------------------------------------------------------------------------------
static void dtw(const float* x, int N, int Mc, int ld, std::vector<int>& ti, std::vector<int>& tj) {
  // the cost matrix as two rolling columns, the trace column-major (the j-outer / i-inner sweep of dtw_cpu then walks
  // contiguous memory), the three-way choice without branches: same comparisons, same tie rule as dtw_cpu
  std::vector<float> colA(N + 1, INFINITY), colB(N + 1, INFINITY);
  std::vector<signed char> tr((size_t)(N + 1) * (Mc + 1), -1);
  auto Tr = [&](int i, int j) -> signed char& { return tr[(size_t)j * (N + 1) + i]; };
  // x transposed to [j][i] in blocks of 16 frames, so the i-inner sweep reads contiguously
  std::vector<float> xt((size_t)Mc * N);
  for (int j0 = 0; j0 < Mc; j0 += 16)
    for (int i = 0; i < N; ++i)
      for (int j = j0; j < std::min(Mc, j0 + 16); ++j) xt[(size_t)j * N + i] = x[(size_t)i * ld + j];
  float* prev = colA.data();  // column j - 1
  float* cur = colB.data();   // column j
  prev[0] = 0.f;              // C(0, 0)
  for (int j = 1; j <= Mc; ++j) {
    cur[0] = INFINITY;  // C(0, j)
    signed char* tcol = &Tr(0, j);
    const float* xj = xt.data() + (size_t)(j - 1) * N;
    float up = cur[0];  // C(i - 1, j)
    for (int i = 1; i <= N; ++i) {
      const float c0 = prev[i - 1], c1 = up, c2 = prev[i];
      const bool p0 = c0 < c1 && c0 < c2, p1 = c1 < c0 && c1 < c2;
      const float v = p0 ? c0 : (p1 ? c1 : c2);
      const signed char t = p0 ? 0 : (p1 ? 1 : 2);
      up = -xj[i - 1] + v;
      cur[i] = up;
      tcol[i] = t;
    }
    std::swap(prev, cur);
  }
  for (int j = 0; j <= Mc; ++j) Tr(0, j) = 2;
  for (int i = 0; i <= N; ++i) Tr(i, 0) = 1;
  int i = N, j = Mc;
  ti.clear();
  tj.clear();
  while (i > 0 || j > 0) {
    ti.push_back(i - 1);
    tj.push_back(j - 1);
    const signed char t = Tr(i, j);
    if (t == 0) {
      --i;
      --j;
    } else if (t == 1) {
      --i;
    } else {
      --j;
    }
  }
  std::reverse(ti.begin(), ti.end());
  std::reverse(tj.begin(), tj.end());
}

// ------------------------------------------------------------------------------------------------
// transcribe
// ------------------------------------------------------------------------------------------------
static void rec(Ctx& c, int i) { WMX_HIP(hipEventRecord(c.ev[i], c.st)); }

static void logmel_dev(Ctx& c, const float* pcm_dev, long stride, const long* lens_host, const int32_t* seek_host, int B,
                       float* out_dev) {
  Model& m = *c.m;
  long maxlen = 0;
  for (int b = 0; b < B; ++b) {
    WMX_CHECK(lens_host[b] >= 0 && lens_host[b] <= c.max_samples && lens_host[b] <= stride, "logmel: bad length");
    maxlen = std::max(maxlen, lens_host[b]);
  }
  std::vector<int> sk(B, 0);
  if (seek_host)
    for (int b = 0; b < B; ++b) sk[b] = seek_host[b];
  WMX_HIP(hipMemcpyAsync(c.lens, lens_host, B * sizeof(long), hipMemcpyHostToDevice, c.st));
  WMX_HIP(hipMemcpyAsync(c.seek, sk.data(), B * 4, hipMemcpyHostToDevice, c.st));
  debug_device("before logmel");
  launch_logmel(pcm_dev, stride, c.lens, c.seek, B, (int)(maxlen / 160) + 1, m.mel_first, m.mel_count, m.mel_off,
                m.mel_w, m.d.n_mels, c.mel_stats, c.mel_stats_cap, out_dev, c.st);
  debug_device("logmel");
  sync(c);  // sk / lens host vectors
}

// rules + selection over c.logits (row_map: logits row of each decode row, NULL = identity) and the greedy / beam
// update that appends the chosen tokens at *slot + 1; with the parity recorder on, the logits and the selection of
// the step are copied out as well
static void select_and_update(Ctx& c, int B, const int* row_map) {
  Model& m = *c.m;
  const int K = c.K, R = K * B;
  const bool rec = c.rec_logits != nullptr;
  if (rec)
    launch_record_logits(c.logits, c.ldl, m.d.n_vocab, R, row_map, c.slot, c.rec_base, c.rec_cap, c.rec_logits, c.st);
  RuleOpts ro{m.d.n_vocab, c.sp.eot, c.sp.timestamp_begin, c.sp.no_timestamps, c.sp.blank, c.o.suppress_blank,
              c.o.max_initial_timestamp_index, c.o.without_timestamps, c.mask};
  ro.err = c.nf_err;
  ro.err_slot = c.slot;
  if (c.sampling) {
    ro.inv_temp = 1.0f / c.o.temperature;
    ro.seed = reinterpret_cast<const uint32_t*>(c.slot + 2);  // written per call (transcribe prologue)
    ro.slot = c.slot;
  }
  launch_logits_select(c.logits, c.ldl, ro, c.rp, R, c.beam ? K + 1 : 1, c.ctok, c.clp, row_map, c.sel_ws, c.st);
  if (!c.beam) {  // greedy, or best_of independent sampled rows
    if (rec) launch_record_select(R, 1, c.ctok, c.rp, c.bs, c.slot, c.rec_base, 0, c.rec_cap, c.rec_sel, c.st);
    launch_greedy_update(c.rp, c.ctok, c.clp, R, c.sp.timestamp_begin, c.sp.eot, c.hist, c.Tctx, c.slot, c.n_done,
                         c.st);
  } else {
    launch_beam_step(c.rp, c.rtmp, c.ctok, c.clp, B, K, c.max_cand, c.sp.timestamp_begin, c.sp.eot, c.slot, c.hist,
                     c.hist_tmp, c.anc, c.anc_tmp, c.Tctx, c.bs, c.n_done, c.st);
    if (rec) launch_record_select(R, K, c.ctok, c.rp, c.bs, c.slot, c.rec_base, 1, c.rec_cap, c.rec_sel, c.st);
  }
}

static void run_step(Ctx& c, int B) {
  // one decode step: forward all rows at slot *slot, select, update (advances *slot)
  Model& m = *c.m;
  FwdArgs f;
  f.rows = c.K * B;
  f.Tn = 1;
  f.rmul = 1;
  f.tok = c.hist;
  f.tok_ld = c.Tctx;
  f.pad_seq = c.pad_row;
  f.prefill = false;
  f.anc = c.beam ? c.anc : nullptr;
  dec_step(c, f);
  dec_logits(c, nullptr, f.rows, true);
  debug_sync(c, "logits", -1);
  select_and_update(c, B, nullptr);
  debug_sync(c, "select_update", -1);
}

// decode steps between n_done read-backs; the chunk is one graph launch
constexpr int kGraphChunk = 8;

static void drop_step_graphs(Ctx& c) {
  for (auto& g : c.graph)
    if (g) {
      (void)hipGraphExecDestroy(g);
      g = nullptr;
    }
  c.graph_key.clear();
}

// capture (once per batch size / rule options / probe placement) a one-step and a kGraphChunk-step graph of
// run_step: every launch reads its step from device state (*slot, histories, ancestry), so a captured step
// replays correctly at any position of the loop, and consecutive captured steps chain on the stream order
static void ensure_step_graphs(Ctx& c, int B) {
  const std::vector<long> key = {B,
                                 c.o.suppress_blank,
                                 c.o.max_initial_timestamp_index,
                                 c.o.without_timestamps,
                                 (long)(intptr_t)c.mask,
                                 (long)(intptr_t)c.rec_logits,
                                 c.probe_kernel,
                                 c.probe_layer};
  if (c.graph[0] && c.graph[1] && key == c.graph_key) return;
  drop_step_graphs(c);
  for (int gi = 0; gi < 2; ++gi) {
    hipGraph_t gph = nullptr;
    WMX_HIP(hipStreamBeginCapture(c.st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < (gi ? kGraphChunk : 1); ++i) run_step(c, B);
    WMX_HIP(hipStreamEndCapture(c.st, &gph));
    WMX_HIP(hipGraphInstantiate(&c.graph[gi], gph, nullptr, nullptr, 0));
    WMX_HIP(hipGraphDestroy(gph));
  }
  c.graph_key = key;
}

// tensors set one by one (wmx_model_set_tensor) since the last preparation: re-derive the MX-fp8, row-major and
// LayerNorm-folded copies before the next use
static void ensure_prepared(Model& m) {
  if (!m.dirty || !m.initialized) return;
  prepare_mx8(m);
  prepare_rowmajor(m);
  prepare_w8(m);
  prepare_fold(m);
  m.dirty = false;
}

static ResultHolder* transcribe(Ctx& c, const float* pcm_dev, long stride, const long* lens, const int32_t* seek, int B,
                                const int32_t* prompt_ids, const int32_t* prompt_lens) {
  Model& m = *c.m;
  WMX_CHECK(m.initialized, "transcribe: model weights not initialised");
  ensure_prepared(m);
  WMX_CHECK(B >= 1 && B <= c.maxB, "transcribe: batch exceeds max_batch");
  const int K = c.K, R = K * B, V = m.d.n_vocab, T = c.Tctx;
  const Special& sp = c.sp;
  // per-call device words: the non-finite guard, and the fused MLP's slice counters + timeout word (zeroed every
  // call, so the monotonic counters never approach 2^32 and a timeout fails only the call it happened in)
  WMX_HIP(hipMemsetAsync(c.nf_err, 0, 4, c.st));
  rec(c, 0);
  logmel_dev(c, pcm_dev, stride, lens, seek, B, c.mel);
  rec(c, 1);
  encode(c, B);
  debug_device("encode");
  rec(c, 2);
  cross_kv(c, B);
  debug_device("cross_kv");
  rec(c, 3);

  // ---- prompts (left padded to Pmax) ----
  std::vector<std::vector<int>> seqs(B);
  const bool detect = c.o.language < 0;
  const int lang_ph = detect ? sp.lang0 : c.o.language;
  const int task_tok = c.o.task == WMX_TASK_TRANSLATE ? sp.translate : sp.transcribe;
  long poff = 0;
  for (int b = 0; b < B; ++b) {
    std::vector<int>& s = seqs[b];
    const int pl = prompt_lens ? prompt_lens[b] : 0;
    if (pl > 0) {
      s.push_back(sp.sot_prev);
      const int keep = std::min(pl, T / 2 - 1);
      for (int i = pl - keep; i < pl; ++i) s.push_back(prompt_ids[poff + i]);
    }
    poff += pl;
    s.push_back(sp.sot);
    s.push_back(lang_ph);
    s.push_back(task_tok);
    if (c.o.without_timestamps) s.push_back(sp.no_timestamps);
  }
  int Pmax = 0;
  for (auto& s : seqs) Pmax = std::max(Pmax, (int)s.size());
  const int sot_tail = c.o.without_timestamps ? 4 : 3;  // sot sits at Pmax - sot_tail
  std::vector<int> hist((size_t)R * T, 0), pad_row(R), pad_win(B), anc((size_t)R * T, 0), lslot(B, Pmax - sot_tail + 1);
  for (int b = 0; b < B; ++b) {
    const int pad = Pmax - (int)seqs[b].size();
    pad_win[b] = pad;
    for (int j = 0; j < K; ++j) {
      const int r = b * K + j;
      pad_row[r] = pad;
      for (size_t i = 0; i < seqs[b].size(); ++i) hist[(size_t)r * T + pad + i] = seqs[b][i];
      for (int s = 0; s < T; ++s) anc[(size_t)r * T + s] = s < Pmax ? b * K : r;
    }
  }
  WMX_HIP(hipMemcpyAsync(c.hist, hist.data(), hist.size() * 4, hipMemcpyHostToDevice, c.st));
  WMX_HIP(hipMemcpyAsync(c.anc, anc.data(), anc.size() * 4, hipMemcpyHostToDevice, c.st));
  WMX_HIP(hipMemcpyAsync(c.pad_row, pad_row.data(), R * 4, hipMemcpyHostToDevice, c.st));
  WMX_HIP(hipMemcpyAsync(c.pad_win, pad_win.data(), B * 4, hipMemcpyHostToDevice, c.st));
  WMX_HIP(hipMemcpyAsync(c.lang_slot, lslot.data(), B * 4, hipMemcpyHostToDevice, c.st));
  // row state reset
  WMX_HIP(hipMemsetAsync(c.rp.ns, 0, R * 4, c.st));
  WMX_HIP(hipMemsetAsync(c.rp.last, 0, R * 4, c.st));
  WMX_HIP(hipMemsetAsync(c.rp.pen, 0, R * 4, c.st));
  WMX_HIP(hipMemsetD32Async((hipDeviceptr_t)c.rp.last_ts, -1, R, c.st));
  WMX_HIP(hipMemsetAsync(c.rp.done, 0, R * 4, c.st));
  WMX_HIP(hipMemsetAsync(c.rp.sum_lp, 0, R * 4, c.st));
  WMX_HIP(hipMemsetAsync(c.bs.win_done, 0, B * 4, c.st));
  WMX_HIP(hipMemsetAsync(c.bs.fin_count, 0, B * 4, c.st));
  WMX_HIP(hipMemsetAsync(c.n_done, 0, 4, c.st));
  std::vector<int> rmap(R);
  for (int r = 0; r < R; ++r) rmap[r] = r / K;
  WMX_HIP(hipMemcpyAsync(c.row_map, rmap.data(), R * 4, hipMemcpyHostToDevice, c.st));
  debug_device("prompt setup");
  sync(c);

  // ---- language detection: one decoder step on <|startoftranscript|> ----
  std::vector<int> lang_out(B, c.o.language);
  std::vector<float> lang_p(B, 1.0f);
  if (detect) {
    // a temporary token row per window: hist_tmp[b*K][0] = sot
    std::vector<int> t1((size_t)B * K * T, sp.sot);
    WMX_HIP(hipMemcpyAsync(c.hist_tmp, t1.data(), t1.size() * 4, hipMemcpyHostToDevice, c.st));
    set_slot(c, 0);
    FwdArgs f;
    f.rows = B;
    f.Tn = 1;
    f.rmul = K;
    f.tok = c.hist_tmp;
    f.tok_ld = (long)K * T;
    f.pad_seq = nullptr;
    f.prefill = true;
    f.anc = nullptr;
    // the split-K decode step, one row per window (it writes cache slot 0 of rows 0 .. B-1, which the prompt
    // prefill rewrites or no hypothesis reads) instead of dec_forward's unsplit projections
    f.win_rows = 1;
    dec_step_fast(c, f);
    dec_logits(c, nullptr, B, true);
    launch_lang_detect(c.logits, c.ldl, sp.lang0, sp.n_langs, B, K, c.hist, T, c.lang_slot, c.lang_tok, c.lang_prob, c.st,
                       c.nf_err);
    debug_sync(c, "lang_detect", -1);
  }
  rec(c, 4);

  // ---- prompt prefill ----
  set_slot(c, 0);
  {
    FwdArgs f;
    f.rows = B;
    f.Tn = Pmax;
    f.rmul = K;
    f.tok = c.hist;
    f.tok_ld = (long)K * T;
    f.pad_seq = c.pad_win;
    f.prefill = true;
    f.anc = nullptr;
    dec_forward(c, f);
    std::vector<int> g(2 * B);
    for (int b = 0; b < B; ++b) {
      g[b] = b * Pmax + Pmax - 1;
      g[B + b] = b * Pmax + Pmax - sot_tail;
    }
    WMX_HIP(hipMemcpyAsync(c.gather, g.data(), g.size() * 4, hipMemcpyHostToDevice, c.st));
    dec_logits(c, c.gather, 2 * B);
    launch_token_prob(c.logits + (size_t)B * c.ldl, c.ldl, V, sp.no_speech, B, c.nospeech, c.st);
    sync(c);
  }
  // this call's sampling seed (slot word 2, read by the captured selection launches)
  if (c.sampling) {
    c.pinned_i[3] = (int)c.o.sample_seed;
    WMX_HIP(hipMemcpyAsync(c.slot + 2, c.pinned_i + 3, 4, hipMemcpyHostToDevice, c.st));
  }
  // first selection from the prefill logits (rows of a window share their window's logits row)
  const int max_new = std::max(0, std::min(c.o.max_new_tokens, T - Pmax));
  set_slot(c, Pmax - 1);
  int steps = 0;
  if (c.rec_logits) {  // recorder step 0 = this first selection (slot Pmax - 1)
    c.rec_R = R;
    c.pinned_i[1] = Pmax - 1;
    WMX_HIP(hipMemcpyAsync(c.rec_base, c.pinned_i + 1, 4, hipMemcpyHostToDevice, c.st));
    WMX_HIP(hipMemsetD32Async((hipDeviceptr_t)c.rec_sel, -1, (size_t)c.rec_cap * c.R * 2, c.st));
    sync(c);
  }
  if (max_new > 0) {
    select_and_update(c, B, c.row_map);
    debug_sync(c, "first_select", -1);
    steps = 1;
  }
  rec(c, 5);
  // ---- decode loop: one hipGraph replay per step ----
  const int need_done = c.beam ? B : R;
  c.probe_slots[0] = steps > 0 ? Pmax : 0;  // slots of the graph-replayed steps of this call

  if (c.probe_kernel >= 0) {  // per-workgroup records of this call only (read after the timed region)
    WMX_HIP(hipMemsetAsync(c.probe_buf, 0, (size_t)kProbeLaunches * T * kProbeWG * 2 * 8, c.st));
  }
  {  // ALGORITHMIC bytes of one launch: weights + activations in + activations out (16-bit), cross K/V
     // (fp8 decode: weights and cross K/V images at 1 byte per element; activations stay 16-bit)
    const double d = m.d.n_text_state, w2 = 2.0, r = R, ww = m.w8 ? 1.0 : 2.0, iw = m.kv8 ? 1.0 : 2.0;
    auto proj = [&](double n, double k) { return n * k * ww + r * k * w2 + r * n * w2; };
    // (fused cross-q: the cross attention also streams the d x d query weights and reads the LN2 rows)
    const bool xqf = c.xq_fused;
    const double xq = xqf ? d * d * ww + r * d * w2 : 0.0;
    const double v[kProbeLaunches] = {proj(3 * d, d), proj(d, d), xqf ? 0.0 : proj(d, d), proj(d, d),
                                      proj(4 * d, d), proj(d, 4 * d), (double)B * 1500 * 2 * d * iw + 2.0 * r * d * w2 + xq};
    for (int k = 0; k < kProbeLaunches; ++k) c.probe_bytes[k] = v[k];
  }
  if (c.o.use_graph && steps < max_new) ensure_step_graphs(c, B);
  if (c.lockstep && steps < max_new) {  // idle stream, then the group's barrier: the step graphs start together
    sync(c);
    c.lockstep_ok = c.lockstep->arrive(std::chrono::microseconds(5000));
  }
  // the group's chunk barrier (default with lockstep; WMX_LOCKSTEP_CHUNKS=0 keeps only the start barrier), left on
  // every exit of the loop
  static const bool lk_every = !(getenv("WMX_LOCKSTEP_CHUNKS") && atoi(getenv("WMX_LOCKSTEP_CHUNKS")) == 0);
  struct LockstepLeave {
    Lockstep* p;
    ~LockstepLeave() {
      if (p) p->leave();
    }
  } lk_leave{c.lockstep && c.lockstep_ok && lk_every && steps < max_new ? c.lockstep.get() : nullptr};
  bool first_chunk = true;
  while (steps < max_new) {
    const int chunk = std::min(kGraphChunk, max_new - steps);
    if (lk_leave.p && !first_chunk && !lk_leave.p->chunk(std::chrono::microseconds(5000))) {
      // a partner more than the timeout behind (or gone): leave the chunk barrier for the rest of this call rather
      // than pay the timeout again at every later chunk
      lk_leave.p->leave();
      lk_leave.p = nullptr;
      ++c.lockstep_timeouts;
    }
    first_chunk = false;
    if (!c.o.use_graph) {
      for (int i = 0; i < chunk; ++i) run_step(c, B);
    } else if (chunk == kGraphChunk) {
      WMX_HIP(hipGraphLaunch(c.graph[1], c.st));  // one launch per chunk: no per-step graph launch bubble
    } else {
      for (int i = 0; i < chunk; ++i) WMX_HIP(hipGraphLaunch(c.graph[0], c.st));
    }
    steps += chunk;
    WMX_HIP(hipMemcpyAsync(c.pinned_i, c.n_done, 4, hipMemcpyDeviceToHost, c.st));
    sync(c);

    if (c.pinned_i[0] >= need_done) break;
  }
  // this member's decode loop is over: release the partners' chunk barriers now, not when transcribe returns
  // (the read-back, the alignment forward and the host DTW below would otherwise hold them at the timeout)
  if (lk_leave.p) {
    lk_leave.p->leave();
    lk_leave.p = nullptr;
  }
  c.last_steps = steps;
  rec(c, 6);
  c.probe_slots[1] = Pmax - 1 + steps;

  // ---- read back and finalise (openai BeamSearchDecoder.finalize + MaximumLikelihoodRanker) ----
  std::vector<int> h((size_t)R * T), ns(R), done(R);
  std::vector<float> slp(R), nosp(B);
  int nf_err = 0;
  WMX_HIP(hipMemcpyAsync(&nf_err, c.nf_err, 4, hipMemcpyDeviceToHost, c.st));
  WMX_HIP(hipMemcpyAsync(h.data(), c.hist, h.size() * 4, hipMemcpyDeviceToHost, c.st));
  WMX_HIP(hipMemcpyAsync(ns.data(), c.rp.ns, R * 4, hipMemcpyDeviceToHost, c.st));
  WMX_HIP(hipMemcpyAsync(done.data(), c.rp.done, R * 4, hipMemcpyDeviceToHost, c.st));
  WMX_HIP(hipMemcpyAsync(slp.data(), c.rp.sum_lp, R * 4, hipMemcpyDeviceToHost, c.st));
  WMX_HIP(hipMemcpyAsync(nosp.data(), c.nospeech, B * 4, hipMemcpyDeviceToHost, c.st));
  if (detect) {
    WMX_HIP(hipMemcpyAsync(lang_out.data(), c.lang_tok, B * 4, hipMemcpyDeviceToHost, c.st));
    WMX_HIP(hipMemcpyAsync(lang_p.data(), c.lang_prob, B * 4, hipMemcpyDeviceToHost, c.st));
  }
  const int nfin = B * c.max_cand;
  std::vector<int> fcount(B), flen(nfin), fh;
  std::vector<float> fscore(nfin);
  if (c.beam) {
    fh.resize((size_t)nfin * T);
    WMX_HIP(hipMemcpyAsync(fcount.data(), c.bs.fin_count, B * 4, hipMemcpyDeviceToHost, c.st));
    WMX_HIP(hipMemcpyAsync(flen.data(), c.bs.fin_len, nfin * 4, hipMemcpyDeviceToHost, c.st));
    WMX_HIP(hipMemcpyAsync(fscore.data(), c.bs.fin_score, nfin * 4, hipMemcpyDeviceToHost, c.st));
    WMX_HIP(hipMemcpyAsync(fh.data(), c.bs.fin_hist, fh.size() * 4, hipMemcpyDeviceToHost, c.st));
  }
  sync(c);
  if (nf_err < 0)
    throw Error(WMX_ERR_NUMERIC, "non-finite decoder logits in language detection, window " + std::to_string(-nf_err - 1));
  if (nf_err != 0) {  // a NaN / inf anywhere upstream of the logits: an error, not a silently shortened transcript
    const int code = nf_err - 1, row = code % 1024, slot = code / 1024;
    throw Error(WMX_ERR_NUMERIC, "non-finite decoder logits at decode step " + std::to_string(slot - (Pmax - 1)) +
                                     " (slot " + std::to_string(slot) + "), row " + std::to_string(row) +
                                     " (window " + std::to_string(row / K) + ")");
  }
  auto* res = new ResultHolder();
  res->data.resize(B);
  res->win.resize(B);
  std::vector<float> sum_lp(B);
  for (int b = 0; b < B; ++b) {
    std::vector<int>& toks = res->data[b].tokens;
    if (K == 1) {
      for (int i = 0; i < ns[b]; ++i) toks.push_back(h[(size_t)b * T + Pmax + i]);
      sum_lp[b] = slp[b];
    } else if (c.sampling) {
      // best_of sampled rows: the highest sum_logprob / length (CT2 sorts its num_hypotheses by that score and
      // faster-whisper takes sequences_ids[0]); ties keep the lower row
      int best = 0;
      double best_score = -INFINITY;
      for (int j = 0; j < K; ++j) {
        const int r = b * K + j;
        const double L = std::max(ns[r], 1);
        const double pen = c.o.length_penalty == 1.0f ? L : std::pow((5.0 + L) / 6.0, (double)c.o.length_penalty);
        const double sc = slp[r] / pen;
        if (sc > best_score) {
          best = j;
          best_score = sc;
        }
      }
      const int r = b * K + best;
      for (int i = 0; i < ns[r]; ++i) toks.push_back(h[(size_t)r * T + Pmax + i]);
      sum_lp[b] = slp[r];
    } else {
      struct Cand {
        std::vector<int> t;
        float s;
      };
      std::vector<Cand> fin;
      for (int f = 0; f < fcount[b]; ++f) {
        const int idx = b * c.max_cand + f;
        Cand cd;
        for (int s = Pmax; s < flen[idx]; ++s) cd.t.push_back(fh[(size_t)idx * T + s]);
        cd.s = fscore[idx];
        fin.push_back(cd);
      }
      if ((int)fin.size() < K) {
        std::vector<int> order(K);
        for (int j = 0; j < K; ++j) order[j] = j;
        std::stable_sort(order.begin(), order.end(),
                         [&](int a, int bb) { return slp[b * K + a] > slp[b * K + bb]; });
        for (int j : order) {
          const int r = b * K + j;
          Cand cd;
          for (int i = 0; i < ns[r]; ++i) cd.t.push_back(h[(size_t)r * T + Pmax + i]);
          cd.s = slp[r];
          bool dup = false;
          for (auto& e : fin) dup = dup || e.t == cd.t;
          if (!dup) fin.push_back(cd);
          if ((int)fin.size() >= K) break;
        }
      }
      int best = -1;
      double best_score = -INFINITY;
      for (size_t i = 0; i < fin.size(); ++i) {
        const double L = std::max<size_t>(fin[i].t.size(), 1);
        const double pen = c.o.length_penalty == 1.0f ? L : std::pow((5.0 + L) / 6.0, (double)c.o.length_penalty);
        const double sc = fin[i].s / pen;
        if (best < 0 || sc > best_score) {
          best = (int)i;
          best_score = sc;
        }
      }
      if (best >= 0) {
        toks = fin[best].t;
        sum_lp[b] = fin[best].s;
      }
    }
    wmx_window_result& w = res->win[b];
    w.language = lang_out[b];
    w.language_prob = lang_p[b];
    w.n_tokens = (int)toks.size();
    w.sum_logprob = sum_lp[b];
    w.avg_logprob = sum_lp[b] / (toks.size() + 1);
    w.no_speech_prob = nosp[b];
    const int F = (int)(lens[b] / 160) + 1;
    const int sk = seek ? seek[b] : 0;
    w.seek_frames = std::max(0, std::min(3000, F - 1 - sk));
  }

  // ---- word alignment: forward sot + text + eot, alignment-head attention -> matrix -> DTW ----
  if (c.o.word_timestamps) {
    std::vector<std::vector<int>> rows(B);
    std::vector<int> ntext(B);
    int Tn = 0;
    for (int b = 0; b < B; ++b) {
      std::vector<int>& s = rows[b];
      // openai timing.find_alignment: sot_sequence + <|notimestamps|> + text tokens + eot
      s = {sp.sot, res->win[b].language, task_tok, sp.no_timestamps};
      for (int t : res->data[b].tokens)
        if (t < sp.eot) s.push_back(t);
      ntext[b] = (int)s.size() - 4;
      s.push_back(sp.eot);
      Tn = std::max(Tn, (int)s.size());
    }
    WMX_CHECK(Tn <= T, "alignment: sequence too long");
    std::vector<int> tok((size_t)B * K * T, 0), ntok(B), nframes(B), target((size_t)B * Tn, -1);
    for (int b = 0; b < B; ++b) {
      for (size_t i = 0; i < rows[b].size(); ++i) tok[(size_t)b * K * T + i] = rows[b][i];
      ntok[b] = (int)rows[b].size();
      nframes[b] = res->win[b].seek_frames;
      for (int i = 0; i < ntext[b]; ++i) target[(size_t)b * Tn + 3 + i] = rows[b][4 + i];
    }
    WMX_HIP(hipMemcpyAsync(c.hist_tmp, tok.data(), tok.size() * 4, hipMemcpyHostToDevice, c.st));
    WMX_HIP(hipMemcpyAsync(c.a_ntok, ntok.data(), B * 4, hipMemcpyHostToDevice, c.st));
    WMX_HIP(hipMemcpyAsync(c.a_nframes, nframes.data(), B * 4, hipMemcpyHostToDevice, c.st));
    WMX_HIP(hipMemcpyAsync(c.a_target, target.data(), target.size() * 4, hipMemcpyHostToDevice, c.st));
    set_slot(c, 0);
    launch_align_matrix_zero(c.align_out, B, Tn, 1500, c.st);
    FwdArgs f;
    f.rows = B;
    f.Tn = Tn;
    f.rmul = K;
    f.tok = c.hist_tmp;
    f.tok_ld = (long)K * T;
    f.pad_seq = nullptr;
    f.prefill = true;
    f.anc = nullptr;
    f.align = true;
    dec_forward(c, f);
    const int nh_total = (int)c.align_heads.size() / 2;
    launch_align_matrix_scale(c.align_out, B, Tn, 1500, c.a_ntok, c.a_nframes, 1.0f / nh_total, c.st);
    // text-token probabilities: logits of every position, in chunks of logits_rows
    const int rows_all = B * Tn;
    for (int r0 = 0; r0 < rows_all; r0 += c.logits_rows) {
      const int n = std::min(c.logits_rows, rows_all - r0);
      std::vector<int> g(n);
      for (int i = 0; i < n; ++i) g[i] = r0 + i;
      WMX_HIP(hipMemcpyAsync(c.gather, g.data(), n * 4, hipMemcpyHostToDevice, c.st));
      dec_logits(c, c.gather, n);
      launch_text_prob(c.logits, c.ldl, sp.eot, c.a_target + r0, n, c.tprob + r0, c.st);
      sync(c);
    }
    c.last_align_ok = false;
    if (!c.h_align) {
      WMX_HIP(hipHostMalloc(&c.h_align, (size_t)c.maxB * c.Tctx * 1500 * sizeof(float)));
      WMX_HIP(hipHostMalloc(&c.h_tp, (size_t)c.maxB * c.Tctx * sizeof(float)));
    }
    float* const mat = c.h_align;  // [B][Tn][1500], pinned
    float* const tp = c.h_tp;
    WMX_HIP(hipMemcpyAsync(mat, c.align_out, (size_t)B * Tn * 1500 * 4, hipMemcpyDeviceToHost, c.st));
    WMX_HIP(hipMemcpyAsync(tp, c.tprob, (size_t)B * Tn * 4, hipMemcpyDeviceToHost, c.st));
    sync(c);
    // DTW per window on host threads
    std::vector<std::thread> th;
    std::atomic<int> next{0};
    const int nth = std::min<int>(B, std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    for (int t = 0; t < nth; ++t)
      th.emplace_back([&]() {
        std::vector<int> ti, tj;
        for (int b = next++; b < B; b = next++) {
          WindowOut& wo = res->data[b];
          const int n = ntext[b] + 1, nf = nframes[b] / 2;
          wo.probs.assign(tp + (size_t)b * Tn + 3, tp + (size_t)b * Tn + 3 + ntext[b]);
          if (nf <= 0) {
            wo.jump_times.assign(n, 0.f);
            continue;
          }
          dtw(mat + ((size_t)b * Tn + 3) * 1500, n, nf, 1500, ti, tj);
          wo.jump_times.clear();
          for (size_t k = 0; k < ti.size(); ++k)
            if (k == 0 || ti[k] != ti[k - 1]) wo.jump_times.push_back(tj[k] / 50.0f);
          wo.jump_times.resize(n, wo.jump_times.empty() ? 0.f : wo.jump_times.back());
        }
      });
    for (auto& x : th) x.join();
    c.last_align_ok = true;  // h_align is read by wmx_ctx_alignment_matrix until the next transcribe
    c.last_ntext = ntext;
    c.last_nframes = nframes;
    c.last_align_Tn = Tn;
  }
  rec(c, 7);
  WMX_HIP(hipEventSynchronize(c.ev[7]));
  for (int i = 0; i < 7; ++i) WMX_HIP(hipEventElapsedTime(&c.stage_ms[i], c.ev[i], c.ev[i + 1]));

  for (int b = 0; b < B; ++b) {
    wmx_window_result& w = res->win[b];
    WindowOut& wo = res->data[b];
    w.tokens = wo.tokens.data();
    w.n_text_tokens = 0;
    for (int t : wo.tokens) w.n_text_tokens += t < sp.eot;
    w.jump_times = wo.jump_times.empty() ? nullptr : wo.jump_times.data();
    w.text_token_probs = wo.probs.empty() ? nullptr : wo.probs.data();
  }
  res->r.n_windows = B;
  res->r.windows = res->win.data();
  return res;
}

}  // namespace wmx

// =================================================================================================
// C ABI
// =================================================================================================
using namespace wmx;

static void free_recorder(Ctx& c) {
  for (void* p : {(void*)c.rec_logits, (void*)c.rec_sel, (void*)c.rec_base})
    if (p) (void)hipFree(p);
  c.rec_logits = nullptr;
  c.rec_sel = nullptr;
  c.rec_base = nullptr;
  c.rec_cap = 0;
}

struct wmx_model {
  Model m;
};
struct wmx_ctx {
  Ctx c;
};

template <class F>
static wmx_status guard(F&& f) {
  try {
    f();
    return WMX_OK;
  } catch (const Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "out of memory";
    return WMX_ERR_NOMEM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return WMX_ERR_STATE;
  }
}

extern "C" {

const char* wmx_last_error(void) { return g_err.c_str(); }
const char* wmx_version(void) { return "wmx 0.1 (gfx950)"; }
int wmx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

wmx_status wmx_model_create(const wmx_dims* dims, int device, int dtype, wmx_model** out) {
  return guard([&] {
    WMX_CHECK(dims && out, "null argument");
    WMX_CHECK(dtype == WMX_DTYPE_BF16 || dtype == WMX_DTYPE_F16 || dtype == WMX_DTYPE_MX8 || dtype == WMX_DTYPE_I8 ||
                  dtype == WMX_DTYPE_I8_BF16,
              "dtype");
    auto* w = new wmx_model();
    try {
      w->m.d = *dims;
      w->m.device = device;
      w->m.dt = (dtype == WMX_DTYPE_F16 || dtype == WMX_DTYPE_I8) ? DT::F16 : DT::BF16;
      w->m.mx8 = dtype == WMX_DTYPE_MX8;
      {  // the fp8 decode of the MX8 model (WMX_DEC_FP8=0: encoder-only MX-fp8, the round-3 model, for A/B runs)
        const char* df = getenv("WMX_DEC_FP8");
        w->m.w8 = w->m.mx8 && !(df && df[0] == '0');
        w->m.kv8 = w->m.w8;
      }
      // the CTranslate2 int8 grid: the 8-bit decode path on int8 bytes + CT2 row scales, 16-bit cross K / V images
      w->m.i8 = dtype == WMX_DTYPE_I8 || dtype == WMX_DTYPE_I8_BF16;
      if (w->m.i8) w->m.w8 = true;
      {  // the mixed decode step, the default for 16-bit models since round 6 (two reduce_ln launches per layer fewer:
         // 439.4-440.4x against the fast step's 416.2-416.8x); WMX_DEC_MIXED=0 selects the fast step
        const char* dm = getenv("WMX_DEC_MIXED");
        w->m.mixed = !w->m.w8 && !(dm && dm[0] == '0');
      }
      {
        const char* ef = getenv("WMX_ENC_FOLD");
        w->m.enc_fold = !w->m.mx8 && w->m.d.n_audio_state % 256 == 0 && !(ef && ef[0] == '0');
      }
      WMX_HIP(hipSetDevice(device));
      WMX_HIP(hipStreamCreateWithFlags(&w->m.st, hipStreamNonBlocking));
      build_model(w->m);
    } catch (...) {
      if (w->m.arena) (void)hipFree(w->m.arena);
      delete w;
      throw;
    }
    *out = w;
  });
}

void wmx_model_free(wmx_model* m) {
  if (!m) return;
  (void)hipSetDevice(m->m.device);
  if (m->m.arena) (void)hipFree(m->m.arena);
  if (m->m.st) (void)hipStreamDestroy(m->m.st);
  delete m;
}

wmx_status wmx_model_init_synthetic(wmx_model* w, uint64_t seed) {
  return guard([&] {
    Model& m = w->m;
    WMX_HIP(hipSetDevice(m.device));
    for (const auto& kv : m.i8_scale_dst)  // (int8 model: every CT2 scale by CT2's rule from the synthetic weights)
      WMX_HIP(hipMemsetAsync(kv.second.first, 0, (size_t)kv.second.second * 4, m.st));
    for (const TensorEntry& e : m.entries) {
      InitSpec s{};
      s.tid = e.tid;
      s.scale = e.scale;
      s.offset = e.offset;
      s.n = e.n;
      s.kind = e.kind;
      s.O = e.O;
      s.C = e.C;
      s.Kp = e.Kp;
      s.dst = e.dst;
      s.store_f32 = e.store_f32;
      launch_init_tensor(m.dt, seed, s, m.st);
    }
    WMX_HIP(hipStreamSynchronize(m.st));
    debug_device("init tensors");
    prepare_mx8(m);
    prepare_rowmajor(m);
    debug_device("prepare_rowmajor");
    prepare_w8(m);
    debug_device("prepare_w8");
    prepare_fold(m);
    debug_device("prepare_fold");
    m.initialized = true;
    m.dirty = false;
  });
}

static const TensorEntry& find_entry(Model& m, const char* name, int64_t n) {
  auto it = m.by_name.find(name);
  WMX_CHECK(it != m.by_name.end(), std::string("unknown tensor ") + name);
  const TensorEntry& e = m.entries[it->second];
  WMX_CHECK(n == e.n, std::string("size mismatch for ") + name);
  return e;
}

wmx_status wmx_model_set_tensor(wmx_model* w, const char* name, const float* data, int64_t n) {
  return guard([&] {
    Model& m = w->m;
    WMX_HIP(hipSetDevice(m.device));
    if (std::string(name) == "encoder.embed_positions.weight") {
      WMX_CHECK(n == 1500L * m.d.n_audio_state, "size mismatch");
      WMX_HIP(hipMemcpy(m.enc_pos, data, n * 4, hipMemcpyHostToDevice));
      return;
    }
    const TensorEntry& e = find_entry(m, name, n);
    m.dirty = true;
    {  // (int8 model: a new weight takes CT2's rule for its scales unless they are set after it)
      const auto it = m.i8_scale_dst.find(name);
      if (it != m.i8_scale_dst.end())
        WMX_HIP(hipMemset(it->second.first, 0, (size_t)it->second.second * 4));
    }
    if (e.store_f32) {
      WMX_HIP(hipMemcpy(e.dst, data, n * 4, hipMemcpyHostToDevice));
      return;
    }
    if (e.kind == 1) {
      std::vector<uint16_t> h((size_t)e.O * e.Kp, 0);
      for (long i = 0; i < n; ++i) {
        const int kk = (int)(i % 3), c = (int)((i / 3) % e.C);
        const long o = i / 3 / e.C;
        h[o * e.Kp + (long)kk * e.C + c] = m.dt == DT::BF16 ? host_f32_to_bf16(data[i]) : host_f32_to_f16(data[i]);
      }
      WMX_HIP(hipMemcpy(e.dst, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    } else if (e.kind == 2) {
      std::vector<uint16_t> h((size_t)(e.O + 15) / 16 * 16 * e.Kp, 0);
      for (long i = 0; i < n; ++i)
        h[packed_index(i / e.Kp, i % e.Kp, e.Kp)] =
            m.dt == DT::BF16 ? host_f32_to_bf16(data[i]) : host_f32_to_f16(data[i]);
      // sub-matrices of fused weights have row counts that are multiples of 16, so h covers exactly their rows
      WMX_HIP(hipMemcpy(e.dst, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    } else {
      std::vector<uint16_t> h(n);
      for (long i = 0; i < n; ++i) h[i] = m.dt == DT::BF16 ? host_f32_to_bf16(data[i]) : host_f32_to_f16(data[i]);
      WMX_HIP(hipMemcpy(e.dst, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    }
  });
}

wmx_status wmx_model_get_tensor(wmx_model* w, const char* name, float* out, int64_t n) {
  return guard([&] {
    Model& m = w->m;
    WMX_HIP(hipSetDevice(m.device));
    WMX_HIP(hipStreamSynchronize(m.st));
    if (std::string(name) == "encoder.embed_positions.weight") {
      WMX_CHECK(n == 1500L * m.d.n_audio_state, "size mismatch");
      WMX_HIP(hipMemcpy(out, m.enc_pos, n * 4, hipMemcpyDeviceToHost));
      return;
    }
    const TensorEntry& e = find_entry(m, name, n);
    m.dirty = true;
    if (e.store_f32) {
      WMX_HIP(hipMemcpy(out, e.dst, n * 4, hipMemcpyDeviceToHost));
      return;
    }
    const long dn = e.kind == 1 ? (long)e.O * e.Kp : (e.kind == 2 ? (long)(e.O + 15) / 16 * 16 * e.Kp : n);
    std::vector<uint16_t> h(dn);
    WMX_HIP(hipMemcpy(h.data(), e.dst, dn * 2, hipMemcpyDeviceToHost));
    for (long i = 0; i < n; ++i) {
      long di = i;
      if (e.kind == 1) {
        const int kk = (int)(i % 3), c = (int)((i / 3) % e.C);
        const long o = i / 3 / e.C;
        di = o * e.Kp + (long)kk * e.C + c;
      } else if (e.kind == 2) {
        di = packed_index(i / e.Kp, i % e.Kp, e.Kp);
      }
      out[i] = m.dt == DT::BF16 ? host_bf16_to_f32(h[di]) : host_f16_to_f32(h[di]);
    }
  });
}

// the CTranslate2 int8 grid (model dtypes I8 / I8_BF16): a decoder projection's (or the token embedding's) CT2 row
// scales, q = rint(w * scale) -- a CT2 int8 checkpoint's weight_scale, set after its weight (reference int8 models:
// 一键实时识别麦克风.py:304, asr_components.py:256-261).  Without it the scales follow CT2's rule 127 / max|row|.
wmx_status wmx_model_set_row_scales(wmx_model* w, const char* name, const float* scale, int64_t n) {
  return guard([&] {
    Model& m = w->m;
    WMX_CHECK(m.i8, "set_row_scales: the model is not an int8 model (WMX_DTYPE_I8 / WMX_DTYPE_I8_BF16)");
    auto it = m.i8_scale_dst.find(name);
    WMX_CHECK(it != m.i8_scale_dst.end(), std::string("set_row_scales: no int8 weight named ") + name);
    WMX_CHECK(n == it->second.second, "set_row_scales: size mismatch");
    for (int64_t i = 0; i < n; ++i)
      WMX_CHECK(std::isfinite(scale[i]) && scale[i] > 0.f, "set_row_scales: scales must be finite and positive");
    WMX_HIP(hipSetDevice(m.device));
    WMX_HIP(hipMemcpy(it->second.first, scale, n * 4, hipMemcpyHostToDevice));
    m.dirty = true;
  });
}

// the device's int8 weights of one such projection (tests: bytes and scales against the checkpoint / CT2's rule):
// q [rows][cols] row-major, scale [rows] the CT2 scales (derived ones included)
wmx_status wmx_model_get_int8(wmx_model* w, const char* name, int8_t* q, float* scale, int64_t rows, int64_t cols) {
  return guard([&] {
    Model& m = w->m;
    WMX_CHECK(m.i8, "get_int8: the model is not an int8 model");
    WMX_HIP(hipSetDevice(m.device));
    ensure_prepared(m);
    auto it = m.i8_scale_dst.find(name);
    WMX_CHECK(it != m.i8_scale_dst.end(), std::string("get_int8: no int8 weight named ") + name);
    WMX_CHECK(rows == it->second.second, "get_int8: rows");
    const int dt = m.d.n_text_state;
    // the 8-bit matrix holding this weight and its first row
    const std::string nm = name;
    const uint8_t* q8 = nullptr;
    long K = dt, r0 = 0, Nall = rows;
    if (nm == "decoder.embed_tokens.weight") {
      q8 = m.tok8;
    } else {
      const int l = std::atoi(nm.c_str() + std::strlen("decoder.layers."));
      const DecLayer& L = m.dec.at(l);
      auto ends = [&](const char* sfx) { return nm.size() > std::strlen(sfx) && nm.compare(nm.size() - std::strlen(sfx), std::string::npos, sfx) == 0; };
      if (ends(".self_attn.q_proj.weight")) q8 = L.q8qkv, r0 = 0, Nall = 3 * dt;
      else if (ends(".self_attn.k_proj.weight")) q8 = L.q8qkv, r0 = dt, Nall = 3 * dt;
      else if (ends(".self_attn.v_proj.weight")) q8 = L.q8qkv, r0 = 2 * dt, Nall = 3 * dt;
      else if (ends(".self_attn.out_proj.weight")) q8 = L.q8o;
      else if (ends(".encoder_attn.q_proj.weight")) q8 = L.q8cq;
      else if (ends(".encoder_attn.out_proj.weight")) q8 = L.q8co;
      else if (ends(".fc1.weight")) q8 = L.q8fc1;
      else if (ends(".fc2.weight")) q8 = L.q8fc2, K = 4 * dt;
    }
    WMX_CHECK(q8 != nullptr && cols == K, "get_int8: shape");
    const long Np = (Nall + 15) / 16 * 16;
    std::vector<uint8_t> h((size_t)Np * K);
    WMX_HIP(hipMemcpy(h.data(), q8, h.size(), hipMemcpyDeviceToHost));
    for (long r = 0; r < rows; ++r)
      for (long k = 0; k < K; ++k) q[r * K + k] = (int8_t)h[packed8_index(r0 + r, k, K)];
    WMX_HIP(hipMemcpy(scale, it->second.first, rows * 4, hipMemcpyDeviceToHost));
  });
}

int64_t wmx_model_n_params(const wmx_model* w) {
  int64_t n = 0;
  for (auto& e : w->m.entries) n += e.n;
  return n;
}

wmx_status wmx_model_arena(wmx_model* w, void** ptr, size_t* bytes) {
  return guard([&] {
    *ptr = w->m.arena;
    *bytes = w->m.param_bytes;  // the parameter region (build_model: the derived copies follow it)
  });
}

wmx_status wmx_model_arena_loaded(wmx_model* w) {
  return guard([&] {
    WMX_HIP(hipSetDevice(w->m.device));
    prepare_mx8(w->m);
    prepare_rowmajor(w->m);
    prepare_w8(w->m);
    prepare_fold(w->m);
    w->m.initialized = true;
    w->m.dirty = false;
  });
}

void wmx_opts_default(wmx_opts* o) {
  std::memset(o, 0, sizeof(*o));
  o->max_batch = 1;
  o->beam_size = 5;
  o->patience = 1.0f;
  o->length_penalty = 1.0f;
  o->max_new_tokens = 448;
  o->task = WMX_TASK_TRANSCRIBE;
  o->language = -1;
  o->without_timestamps = 0;
  o->max_initial_timestamp_index = 50;
  o->suppress_blank = 1;
  o->word_timestamps = 1;
  o->median_filter_width = 7;
  o->use_graph = 1;
  o->max_audio_samples = 480000;
  o->temperature = 0.0f;
  o->best_of = 5;
  o->sample_seed = 0;
}

wmx_status wmx_ctx_create(wmx_model* w, const wmx_opts* o, wmx_ctx** out) {
  return guard([&] {
    WMX_CHECK(w && o && out, "null argument");
    // round 5's timing-only launch ablation (results wrong by construction) was removed from the library; a stale
    // WMX_ABLATE in the environment fails loudly rather than suggesting that a product run measured it
    WMX_CHECK(getenv("WMX_ABLATE") == nullptr, "WMX_ABLATE is set: the timing-only decode ablation was removed (unset it)");
    WMX_CHECK(o->max_batch >= 1 && o->beam_size >= 1 && o->beam_size <= 8, "opts: batch / beam");
    WMX_CHECK(o->temperature >= 0.f && std::isfinite(o->temperature), "opts: temperature");
    WMX_CHECK(o->temperature == 0.f || (o->best_of >= 1 && o->best_of <= 8), "opts: best_of (1..8) when sampling");
    const int rows_per_win = o->temperature > 0.f ? o->best_of : o->beam_size;
    WMX_CHECK(rows_per_win * o->max_batch <= 1024, "opts: rows per window * batch <= 1024");
    WMX_CHECK(o->median_filter_width >= 1 && o->median_filter_width <= 15 && o->median_filter_width % 2 == 1,
              "opts: median_filter_width");
    WMX_HIP(hipSetDevice(w->m.device));
    auto* x = new wmx_ctx();
    Ctx& c = x->c;
    try {
      c.m = &w->m;
      c.o = *o;
      c.dt = w->m.dt;
      c.maxB = o->max_batch;
      c.sampling = o->temperature > 0.f;
      c.K = rows_per_win;
      c.beam = !c.sampling && c.K > 1;
      c.R = c.K * c.maxB;
      c.Tctx = w->m.d.n_text_ctx;
      c.max_samples = o->max_audio_samples > 0 ? o->max_audio_samples : 480000;
      c.sp = Special(w->m.d.n_vocab);
      if (o->suppress_tokens && o->n_suppress_tokens > 0)
        c.suppress.assign(o->suppress_tokens, o->suppress_tokens + o->n_suppress_tokens);
      const int Lt = w->m.d.n_text_layer, Ht = w->m.d.n_text_head;
      if (o->alignment_heads && o->n_alignment_heads > 0) {
        c.align_heads.assign(o->alignment_heads, o->alignment_heads + 2 * o->n_alignment_heads);
        for (size_t i = 0; i + 1 < c.align_heads.size(); i += 2)
          WMX_CHECK(c.align_heads[i] >= 0 && c.align_heads[i] < Lt && c.align_heads[i + 1] >= 0 &&
                        c.align_heads[i + 1] < Ht,
                    "opts: alignment head out of range");
      } else {
        for (int l = Lt / 2; l < Lt; ++l)
          for (int h = 0; h < Ht; ++h) {
            c.align_heads.push_back(l);
            c.align_heads.push_back(h);
          }
      }
      c.o.suppress_tokens = nullptr;
      c.o.alignment_heads = nullptr;
      WMX_HIP(hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking));
      // fused cross-q is the default (397-398 vs 383-384x real time, gpurun_out/r02za); WMX_XQ_FUSED=0 restores the
      // separate split-K launch (A/B runs)
      // (the int8 model: the cross-q projection on its int8 weights, its own launch -- the fused 8-bit query
      // projection reads e4m3 weights beside fp8 images only)
      c.xq_fused = !(getenv("WMX_XQ_FUSED") && atoi(getenv("WMX_XQ_FUSED")) == 0) && !w->m.i8;
      gemm_init_attributes();
      alloc_ctx(c);
    } catch (...) {
      if (c.buf) (void)hipFree(c.buf);
      if (c.dsp_scratch) (void)hipFree(c.dsp_scratch);
      if (c.dsp_io) (void)hipFree(c.dsp_io);
      if (c.dsp_lens) (void)hipFree(c.dsp_lens);
      for (void* p : {(void*)c.pinned_i, (void*)c.h_align, (void*)c.h_tp})
        if (p) (void)hipHostFree(p);
      if (c.st) (void)hipStreamDestroy(c.st);
      delete x;
      throw;
    }
    *out = x;
  });
}

void wmx_ctx_destroy(wmx_ctx* x) {
  if (!x) return;
  Ctx& c = x->c;
  (void)hipSetDevice(c.m->device);
  (void)hipStreamSynchronize(c.st);
  drop_step_graphs(c);
  free_recorder(c);
  if (c.buf) (void)hipFree(c.buf);
  if (c.pinned_i) (void)hipHostFree(c.pinned_i);
  if (c.h_align) (void)hipHostFree(c.h_align);
  if (c.h_tp) (void)hipHostFree(c.h_tp);
  for (auto& e : c.ev)
    if (e) (void)hipEventDestroy(e);
  if (c.st) (void)hipStreamDestroy(c.st);
  delete x;
}

void* wmx_ctx_stream(wmx_ctx* x) { return (void*)x->c.st; }

wmx_status wmx_logmel_device(wmx_ctx* x, const float* pcm_dev, int64_t stride, const int64_t* lens, const int32_t* seek,
                             int B, float* mel_out_dev) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(B >= 1 && B <= c.maxB, "logmel: batch");
    WMX_HIP(hipSetDevice(c.m->device));
    std::vector<long> l(lens, lens + B);
    logmel_dev(c, pcm_dev, (long)stride, l.data(), seek, B, mel_out_dev);
  });
}

wmx_status wmx_logmel(wmx_ctx* x, const float* pcm, int64_t stride, const int64_t* lens, const int32_t* seek, int B,
                      float* mel_out) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(B >= 1 && B <= c.maxB, "logmel: batch");
    WMX_CHECK(stride <= c.max_samples, "logmel: stride exceeds max_audio_samples");
    WMX_HIP(hipSetDevice(c.m->device));
    WMX_HIP(hipMemcpyAsync(c.pcm, pcm, (size_t)B * stride * 4, hipMemcpyHostToDevice, c.st));
    std::vector<long> l(lens, lens + B);
    logmel_dev(c, c.pcm, (long)stride, l.data(), seek, B, c.mel);
    WMX_HIP(hipMemcpyAsync(mel_out, c.mel, (size_t)B * c.m->d.n_mels * 3000 * 4, hipMemcpyDeviceToHost, c.st));
    sync(c);
  });
}

wmx_status wmx_encode_device(wmx_ctx* x, const float* mel_dev, int B) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(c.m->initialized, "encode: weights not initialised");
    WMX_CHECK(B >= 1 && B <= c.maxB, "encode: batch");
    WMX_HIP(hipSetDevice(c.m->device));
    ensure_prepared(*c.m);
    if (mel_dev != c.mel)
      WMX_HIP(hipMemcpyAsync(c.mel, mel_dev, (size_t)B * c.m->d.n_mels * 3000 * 4, hipMemcpyDeviceToDevice, c.st));
    encode(c, B);
    cross_kv(c, B);
    sync(c);
  });
}

wmx_status wmx_encode(wmx_ctx* x, const float* mel, int B, float* enc_out) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(c.m->initialized, "encode: weights not initialised");
    WMX_CHECK(B >= 1 && B <= c.maxB, "encode: batch");
    WMX_HIP(hipSetDevice(c.m->device));
    ensure_prepared(*c.m);
    WMX_HIP(hipMemcpyAsync(c.mel, mel, (size_t)B * c.m->d.n_mels * 3000 * 4, hipMemcpyHostToDevice, c.st));
    encode(c, B);
    cross_kv(c, B);
    if (enc_out) {
      const long n = (long)B * 1500 * c.m->d.n_audio_state;
      launch_cvt16_to_f32(c.dt, c.enc_out, c.ex, n, c.st);
      WMX_HIP(hipMemcpyAsync(enc_out, c.ex, n * 4, hipMemcpyDeviceToHost, c.st));
    }
    sync(c);
  });
}

wmx_status wmx_decoder_logits(wmx_ctx* x, const int32_t* tokens, const int32_t* lens, int B, int T, float* logits_out) {
  return guard([&] {
    Ctx& c = x->c;
    Model& m = *c.m;
    WMX_CHECK(B >= 1 && B <= c.maxB && T >= 1 && T <= c.Tctx, "decoder_logits: shape");
    ensure_prepared(m);
    WMX_HIP(hipSetDevice(m.device));
    const int K = c.K, Tc = c.Tctx, V = m.d.n_vocab;
    std::vector<int> tok((size_t)B * K * Tc, 0);
    for (int b = 0; b < B; ++b)
      for (int i = 0; i < T; ++i) tok[(size_t)b * K * Tc + i] = tokens[(size_t)b * T + i];
    WMX_HIP(hipMemcpyAsync(c.hist_tmp, tok.data(), tok.size() * 4, hipMemcpyHostToDevice, c.st));
    set_slot(c, 0);
    FwdArgs f;
    f.rows = B;
    f.Tn = T;
    f.rmul = K;
    f.tok = c.hist_tmp;
    f.tok_ld = (long)K * Tc;
    f.pad_seq = nullptr;
    f.prefill = true;
    f.anc = nullptr;
    dec_forward(c, f);
    const int rows_all = B * T;
    for (int r0 = 0; r0 < rows_all; r0 += c.logits_rows) {
      const int n = std::min(c.logits_rows, rows_all - r0);
      std::vector<int> g(n);
      for (int i = 0; i < n; ++i) g[i] = r0 + i;
      WMX_HIP(hipMemcpyAsync(c.gather, g.data(), n * 4, hipMemcpyHostToDevice, c.st));
      dec_logits(c, c.gather, n);
      WMX_HIP(hipMemcpy2DAsync(logits_out + (size_t)r0 * V, (size_t)V * 4, c.logits, (size_t)c.ldl * 4, (size_t)V * 4, n,
                               hipMemcpyDeviceToHost, c.st));
      sync(c);
    }
    (void)lens;
  });
}

wmx_status wmx_ctx_forced_decode(wmx_ctx* x, const int32_t* prefix, const int32_t* prefix_lens, int P, int B,
                                 int n_steps, const int32_t* tokens, const int32_t* parents, int32_t* top1,
                                 float* logits, int every) {
  return guard([&] {
    Ctx& c = x->c;
    Model& m = *c.m;
    WMX_CHECK(m.initialized, "forced_decode: weights not initialised");
    ensure_prepared(m);
    WMX_CHECK(B >= 1 && B <= c.maxB && P >= 1 && n_steps >= 0 && P + n_steps <= c.Tctx, "forced_decode: shape");
    WMX_CHECK(prefix && top1 && (n_steps == 0 || (tokens && parents)) && (!logits || every >= 1),
              "forced_decode: null argument");
    WMX_HIP(hipSetDevice(m.device));
    const int K = c.K, R = K * B, T = c.Tctx, V = m.d.n_vocab;
    for (int i = 0; i < n_steps; ++i)
      for (int r = 0; r < R; ++r) {
        const int p = parents[(size_t)i * R + r], t = tokens[(size_t)i * R + r];
        WMX_CHECK(p >= 0 && p < R && p / K == r / K, "forced_decode: parent outside the row's window");
        WMX_CHECK(t >= 0 && t < V, "forced_decode: token id");
      }
    // the layout transcribe() sets up: window b's prefix (prefix_lens[b] ids) left-padded to P; row r of window b
    // holds it, and its slots < P live in cache row b*K
    std::vector<int> hist((size_t)R * T, 0), anc((size_t)R * T, 0), pad_row(R), pad_win(B);
    for (int b = 0; b < B; ++b) {
      const int n = prefix_lens ? prefix_lens[b] : P;
      WMX_CHECK(n >= 1 && n <= P, "forced_decode: prefix length");
      pad_win[b] = P - n;
    }
    for (int r = 0; r < R; ++r) {
      const int b = r / K;
      pad_row[r] = pad_win[b];
      for (int i = pad_win[b]; i < P; ++i) hist[(size_t)r * T + i] = prefix[(size_t)b * P + i - pad_win[b]];
      for (int s = 0; s < T; ++s) anc[(size_t)r * T + s] = s < P ? b * K : r;
    }
    WMX_HIP(hipMemcpyAsync(c.hist, hist.data(), hist.size() * 4, hipMemcpyHostToDevice, c.st));
    WMX_HIP(hipMemcpyAsync(c.pad_row, pad_row.data(), R * 4, hipMemcpyHostToDevice, c.st));
    WMX_HIP(hipMemcpyAsync(c.pad_win, pad_win.data(), B * 4, hipMemcpyHostToDevice, c.st));
    set_slot(c, 0);
    std::vector<float> lg((size_t)R * V);
    auto collect = [&](int step, int nrows, int rep) {  // logits rows [0, nrows) -> top1 / logits of R rows
      WMX_HIP(hipMemcpy2DAsync(lg.data(), (size_t)V * 4, c.logits, (size_t)c.ldl * 4, (size_t)V * 4, nrows,
                               hipMemcpyDeviceToHost, c.st));
      sync(c);
      for (int r = 0; r < R; ++r) {
        const float* row = lg.data() + (size_t)(r / rep) * V;
        int best = 0;
        for (int v = 1; v < V; ++v)
          if (row[v] > row[best]) best = v;
        top1[(size_t)step * R + r] = best;
        if (logits && step % every == 0)
          std::memcpy(logits + ((size_t)(step / every) * R + r) * V, row, (size_t)V * 4);
      }
    };
    {  // prefill of the prefix, one sequence per window (cache rows b*K), logits of its last position
      FwdArgs f;
      f.rows = B;
      f.Tn = P;
      f.rmul = K;
      f.tok = c.hist;
      f.tok_ld = (long)K * T;
      f.pad_seq = c.pad_win;
      f.prefill = true;
      f.anc = nullptr;
      dec_forward(c, f);
      std::vector<int> g(B);
      for (int b = 0; b < B; ++b) g[b] = b * P + P - 1;
      WMX_HIP(hipMemcpyAsync(c.gather, g.data(), B * 4, hipMemcpyHostToDevice, c.st));
      dec_logits(c, c.gather, B);
      collect(0, B, K);
    }
    std::vector<int> h2(hist.size()), a2(anc.size());
    for (int i = 0; i < n_steps; ++i) {
      const int s = P - 1 + i;  // slot of the last history token; the forced token goes to s + 1
      for (int r = 0; r < R; ++r) {  // beam_update_kernel: parent history + ancestry, new token, own cache row
        const int p = parents[(size_t)i * R + r];
        std::memcpy(&h2[(size_t)r * T], &hist[(size_t)p * T], (size_t)T * 4);
        std::memcpy(&a2[(size_t)r * T], &anc[(size_t)p * T], (size_t)T * 4);
        h2[(size_t)r * T + s + 1] = tokens[(size_t)i * R + r];
        a2[(size_t)r * T + s + 1] = r;
      }
      hist.swap(h2);
      anc.swap(a2);
      WMX_HIP(hipMemcpyAsync(c.hist, hist.data(), hist.size() * 4, hipMemcpyHostToDevice, c.st));
      WMX_HIP(hipMemcpyAsync(c.anc, anc.data(), anc.size() * 4, hipMemcpyHostToDevice, c.st));
      set_slot(c, s + 1);
      // the launches of run_step() before its selection
      FwdArgs f;
      f.rows = R;
      f.Tn = 1;
      f.rmul = 1;
      f.tok = c.hist;
      f.tok_ld = T;
      f.pad_seq = c.pad_row;
      f.prefill = false;
      f.anc = c.beam ? c.anc : nullptr;
      dec_step(c, f);
      dec_logits(c, nullptr, R, true);
      collect(i + 1, R, 1);
    }
  });
}

wmx_status wmx_debug_packed_launch(int M, int N, int K, int64_t part_cap, int split, int64_t lda, int64_t* out9) {
  return guard([&] {
    WMX_CHECK(out9 && M >= 1 && N >= 1 && K >= 32 && K % 32 == 0, "debug_packed_launch: arguments");
    // the split count the runtime's callers use: gemm_p (S = 1, epilogue) or gemm_p_part (partials, S >= 2)
    int S = 1;
    if (split == 1) {
      S = packed_splits(M, N, K, part_cap);
      if (S == 1) S = 2;
    }
    const int nct = split == 2 ? 1 : 0;  // 2: the unsplit residual producers of the folded step (gemm_p_resid)
    const PackedPlan p = packed_plan(M, N, K, S, nct);
    const PackedExtent e = packed_extent(M, N, K, S, lda, nct);
    const int64_t v[9] = {S, p.MT, p.NCT, p.NW, p.KU, e.w_end, e.a_end, e.part_end, e.stray_ksteps};
    std::memcpy(out9, v, sizeof(v));
  });
}

// debug (WMX_GUARD=1 at creation): the first guard gap of the model / context arena whose pattern was overwritten:
// *model_buf / *ctx_buf = the index (in planner add order) of the buffer it follows, -1 when intact
static int guard_scan(const char* base, const std::vector<std::pair<size_t, size_t>>& g, hipStream_t st) {
  std::vector<unsigned char> h;
  WMX_HIP(hipStreamSynchronize(st));
  for (size_t i = 0; i < g.size(); ++i) {
    h.resize(g[i].second);
    WMX_HIP(hipMemcpy(h.data(), base + g[i].first, g[i].second, hipMemcpyDeviceToHost));
    for (unsigned char v : h)
      if (v != 0xA5) return (int)i;
  }
  return -1;
}
wmx_status wmx_debug_guard_check(wmx_model* w, wmx_ctx* x, int* model_buf, int* ctx_buf) {
  return guard([&] {
    WMX_CHECK(model_buf && ctx_buf, "guard_check: null argument");
    *model_buf = w ? guard_scan(w->m.arena, w->m.guards, w->m.st) : -1;
    *ctx_buf = x ? guard_scan(x->c.buf, x->c.guards, x->c.st) : -1;
  });
}

// the shader-clock probe beside a workload: start launches it on a stream of its own and returns; result waits
// for it and copies the n per-workgroup clocks (MHz)
static struct {
  hipStream_t st = nullptr;
  float* buf = nullptr;
  int n = 0, device = -1;
} g_clock;

wmx_status wmx_debug_clock_start(int device, double ms, int n) {
  return guard([&] {
    WMX_CHECK(ms > 0 && ms <= 10000 && n >= 1 && n <= 256 && g_clock.n == 0, "clock_start: arguments / pending probe");
    WMX_HIP(hipSetDevice(device));
    if (g_clock.device != device) {
      if (g_clock.st) (void)hipStreamDestroy(g_clock.st);
      if (g_clock.buf) (void)hipFree(g_clock.buf);
      g_clock.st = nullptr;
      g_clock.buf = nullptr;
      WMX_HIP(hipStreamCreateWithFlags(&g_clock.st, hipStreamNonBlocking));
      WMX_HIP(hipMalloc((void**)&g_clock.buf, 256 * sizeof(float)));
      g_clock.device = device;
    }
    launch_clock_probe(g_clock.buf, n, ms, g_clock.st);
    g_clock.n = n;
  });
}

wmx_status wmx_debug_clock_result(float* mhz, int n) {
  return guard([&] {
    WMX_CHECK(mhz && g_clock.n > 0 && n == g_clock.n, "clock_result: no probe pending / count");
    WMX_HIP(hipSetDevice(g_clock.device));
    g_clock.n = 0;
    WMX_HIP(hipStreamSynchronize(g_clock.st));
    WMX_HIP(hipMemcpy(mhz, g_clock.buf, n * sizeof(float), hipMemcpyDeviceToHost));
  });
}

wmx_status wmx_debug_dtw(const float* x, int N, int M, int ld, int32_t* ti, int32_t* tj, int* len) {
  return guard([&] {
    WMX_CHECK(x && ti && tj && len && N >= 1 && M >= 1 && ld >= M, "debug_dtw: arguments");
    std::vector<int> a, b;
    dtw(x, N, M, ld, a, b);
    const int n = (int)a.size();
    for (int k = 0; k < n; ++k) {  // path order, as dtw() leaves it
      ti[k] = a[k];
      tj[k] = b[k];
    }
    *len = n;
  });
}

wmx_status wmx_ctx_record(wmx_ctx* x, int max_steps) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(max_steps >= 0 && max_steps <= c.Tctx, "record: max_steps");
    WMX_HIP(hipSetDevice(c.m->device));
    sync(c);
    drop_step_graphs(c);  // the captured steps carry (or lack) the record launches
    free_recorder(c);
    if (max_steps == 0) return;
    WMX_HIP(hipMalloc(&c.rec_logits, (size_t)max_steps * c.R * c.m->d.n_vocab * 4));
    WMX_HIP(hipMalloc(&c.rec_sel, (size_t)max_steps * c.R * 2 * 4));
    WMX_HIP(hipMalloc(&c.rec_base, 4));
    c.rec_cap = max_steps;
  });
}

wmx_status wmx_ctx_recorded(wmx_ctx* x, float* logits, int32_t* sel, int* n_steps, int* rows) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(c.rec_logits, "recorded: the recorder is off (wmx_ctx_record)");
    WMX_CHECK(n_steps && rows, "recorded: null argument");
    WMX_HIP(hipSetDevice(c.m->device));
    const int n = std::min(c.last_steps, c.rec_cap);
    *n_steps = n;
    *rows = c.rec_R;
    if (logits)
      WMX_HIP(hipMemcpy(logits, c.rec_logits, (size_t)n * c.rec_R * c.m->d.n_vocab * 4, hipMemcpyDeviceToHost));
    if (sel) WMX_HIP(hipMemcpy(sel, c.rec_sel, (size_t)n * c.rec_R * 2 * 4, hipMemcpyDeviceToHost));
  });
}

wmx_status wmx_ctx_set_sample_seed(wmx_ctx* x, uint32_t seed) {
  return guard([&] { x->c.o.sample_seed = seed; });
}

wmx_status wmx_ctx_alignment_matrix(wmx_ctx* x, int b, float* out, int* n, int* nf) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(n && nf, "alignment_matrix: null argument");
    WMX_CHECK(c.last_align_ok && b >= 0 && b < (int)c.last_ntext.size(),
              "alignment_matrix: no word alignment for this window in the last transcribe");
    const int rows = c.last_ntext[b] + 1, cols = c.last_nframes[b] / 2;
    *n = rows;
    *nf = cols;
    if (!out) return;
    for (int i = 0; i < rows; ++i)
      std::memcpy(out + (size_t)i * cols, c.h_align + ((size_t)b * c.last_align_Tn + 3 + i) * 1500,
                  (size_t)std::max(cols, 0) * 4);
  });
}

wmx_status wmx_transcribe_device(wmx_ctx* x, const float* pcm_dev, int64_t stride, const int64_t* lens,
                                 const int32_t* seek, int B, const int32_t* prompt_ids, const int32_t* prompt_lens,
                                 wmx_result** out) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(out, "null out");
    WMX_HIP(hipSetDevice(c.m->device));
    std::vector<long> l(lens, lens + B);
    ResultHolder* r = transcribe(c, pcm_dev, (long)stride, l.data(), seek, B, prompt_ids, prompt_lens);
    *out = &r->r;
  });
}

wmx_status wmx_transcribe(wmx_ctx* x, const float* pcm, int64_t stride, const int64_t* lens, const int32_t* seek, int B,
                          const int32_t* prompt_ids, const int32_t* prompt_lens, wmx_result** out) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(out, "null out");
    WMX_CHECK(B >= 1 && B <= c.maxB, "transcribe: batch");
    WMX_CHECK(stride <= c.max_samples, "transcribe: stride exceeds max_audio_samples");
    WMX_HIP(hipSetDevice(c.m->device));
    WMX_HIP(hipMemcpyAsync(c.pcm, pcm, (size_t)B * stride * 4, hipMemcpyHostToDevice, c.st));
    std::vector<long> l(lens, lens + B);
    ResultHolder* r = transcribe(c, c.pcm, (long)stride, l.data(), seek, B, prompt_ids, prompt_lens);
    *out = &r->r;
  });
}

void wmx_result_free(wmx_result* r) {
  if (!r) return;
  // r is the first member of ResultHolder
  delete reinterpret_cast<ResultHolder*>(r);
}

wmx_status wmx_ctx_stage_ms(wmx_ctx* x, float* out7) {
  return guard([&] { std::memcpy(out7, x->c.stage_ms, sizeof(float) * 7); });
}

int wmx_ctx_last_steps(wmx_ctx* x) { return x->c.last_steps; }
wmx_status wmx_ctx_lockstep_timeouts(wmx_ctx* x, int64_t* n) {
  if (!x || !n) return WMX_ERR_ARG;
  *n = (int64_t)x->c.lockstep_timeouts;
  return WMX_OK;
}

// ---- pre-ASR DSP ----
static void grow_bytes(void** p, size_t& cap, size_t need, size_t elem) {
  if (need <= cap) return;
  if (*p) WMX_HIP(hipFree(*p));
  *p = nullptr;
  WMX_HIP(hipMalloc(p, need * elem));
  cap = need;
}

static void dsp_lens_upload(Ctx& c, const int64_t* lens, int B) {
  if (B > c.dsp_lens_cap) {
    if (c.dsp_lens) WMX_HIP(hipFree(c.dsp_lens));
    c.dsp_lens = nullptr;
    WMX_HIP(hipMalloc(&c.dsp_lens, (size_t)B * sizeof(long)));
    c.dsp_lens_cap = B;
  }
  std::vector<long> l(lens, lens + B);
  WMX_HIP(hipMemcpyAsync(c.dsp_lens, l.data(), (size_t)B * sizeof(long), hipMemcpyHostToDevice, c.st));
  sync(c);  // l goes out of scope
}

static void filtfilt_dev(Ctx& c, const float* x, long stride, const int64_t* lens, int B, const double* b,
                         const double* a, const double* zi, int ntaps, float* y) {
  WMX_CHECK(B >= 1 && ntaps >= 2 && ntaps <= kMaxTaps, "filtfilt: batch / filter order");
  IIRCoefs f{};
  for (int i = 0; i < ntaps; ++i) {
    f.b[i] = b[i];
    f.a[i] = a[i];
  }
  for (int i = 0; i + 1 < ntaps; ++i) f.zi[i] = zi[i];
  f.ntaps = ntaps;
  f.padlen = 3 * ntaps;
  long mx = 0;
  for (int i = 0; i < B; ++i) {
    WMX_CHECK(lens[i] >= 0 && lens[i] <= stride, "filtfilt: length exceeds stride");
    WMX_CHECK(lens[i] == 0 || lens[i] > f.padlen, "filtfilt: input shorter than padlen (scipy raises)");
    mx = std::max<long>(mx, lens[i]);
  }
  const long sstride = mx + 2L * f.padlen;
  grow_bytes((void**)&c.dsp_scratch, c.dsp_scratch_elems, (size_t)B * sstride, sizeof(double));
  dsp_lens_upload(c, lens, B);
  launch_filtfilt(x, stride, c.dsp_lens, B, f, c.dsp_scratch, sstride, y, stride, c.st);
}

wmx_status wmx_filtfilt_device(wmx_ctx* x, const float* x_dev, int64_t stride, const int64_t* lens, int B,
                               const double* b, const double* a, const double* zi, int ntaps, float* y_dev) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_HIP(hipSetDevice(c.m->device));
    filtfilt_dev(c, x_dev, (long)stride, lens, B, b, a, zi, ntaps, y_dev);
    sync(c);
  });
}

wmx_status wmx_filtfilt(wmx_ctx* x, const float* xh, int64_t stride, const int64_t* lens, int B, const double* b,
                        const double* a, const double* zi, int ntaps, float* y) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_HIP(hipSetDevice(c.m->device));
    WMX_CHECK(B >= 1 && stride >= 1, "filtfilt: batch");
    const size_t n = (size_t)B * stride;
    grow_bytes((void**)&c.dsp_io, c.dsp_io_elems, 2 * n, sizeof(float));
    WMX_HIP(hipMemcpyAsync(c.dsp_io, xh, n * 4, hipMemcpyHostToDevice, c.st));
    filtfilt_dev(c, c.dsp_io, (long)stride, lens, B, b, a, zi, ntaps, c.dsp_io + n);
    WMX_HIP(hipMemcpyAsync(y, c.dsp_io + n, n * 4, hipMemcpyDeviceToHost, c.st));
    sync(c);
  });
}

wmx_status wmx_dedup_features(wmx_ctx* x, const float* xh, int64_t stride, const int64_t* lens, int B, float sr,
                              float* out) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_HIP(hipSetDevice(c.m->device));
    WMX_CHECK(B >= 1 && stride >= 1 && sr > 0, "dedup features: batch / rate");
    for (int i = 0; i < B; ++i)
      WMX_CHECK(lens[i] >= 0 && lens[i] <= stride && lens[i] <= kDedupMaxN, "dedup features: chunk length");
    const size_t n = (size_t)B * stride;
    grow_bytes((void**)&c.dsp_io, c.dsp_io_elems, n + (size_t)B * 5, sizeof(float));
    WMX_HIP(hipMemcpyAsync(c.dsp_io, xh, n * 4, hipMemcpyHostToDevice, c.st));
    dsp_lens_upload(c, lens, B);
    launch_dedup_features(c.dsp_io, (long)stride, c.dsp_lens, B, sr, c.dsp_io + n, c.st);
    WMX_HIP(hipMemcpyAsync(out, c.dsp_io + n, (size_t)B * 5 * 4, hipMemcpyDeviceToHost, c.st));
    sync(c);
  });
}

wmx_status wmx_ctx_set_probe(wmx_ctx* x, int kernel, int layer) {
  return guard([&] {
    WMX_CHECK(kernel < 1, "probe: 0 enables the decode-step probes, < 0 disables them");
    WMX_CHECK(layer >= 1 && layer < x->c.m->d.n_text_layer, "probe: layer (>= 1: the previous layer is probed too)");
    Ctx& c = x->c;
    c.probe_kernel = kernel;
    c.probe_layer = layer;
  });
}

// per probed launch id, averaged over the decode steps of the last transcribe: span = latest workgroup end -
// earliest workgroup start (execution only); e2e = its latest workgroup end - that of the launch before it in the
// layer's chain (dispatch + execution: the per-kernel span rocprofv3 reports, plus the inter-kernel gap)
static void probe_collect(Ctx& c, double* ms, int* n, double* e2e, int* e2e_n) {
  const int T = c.Tctx;
  std::vector<unsigned long long> tk((size_t)kProbeLaunches * T * kProbeWG * 2);
  WMX_HIP(hipStreamSynchronize(c.st));
  WMX_HIP(hipMemcpy(tk.data(), c.probe_buf, tk.size() * 8, hipMemcpyDeviceToHost));
  // the chain of one layer's launches (dec_step_fast / dec_step_mixed)
  static const int chain_fast[] = {kProbePrev, kProbeQKV, kProbeSelf, kProbeOut, kProbeRedOut, kProbeCrossQ,
                                   kProbeCross, kProbeCrossOut, kProbeRedCrossOut, kProbeFc1, kProbeFc2, kProbeRedFc2};
  static const int chain_mixed[] = {kProbePrev, kProbeQKV, kProbeSelf, kProbeOut, kProbeCross, kProbeCrossOut,
                                    kProbeFc1, kProbeFc2, kProbeRedFc2};
  const bool mixed = c.m->mixed && c.xq_fused;
  const int* chain = mixed ? chain_mixed : chain_fast;
  const int nchain = mixed ? 9 : 12;
  for (int k = 0; k < kProbeLaunches; ++k) {
    ms[k] = e2e[k] = 0;
    n[k] = e2e_n[k] = 0;
  }
  for (int sl = c.probe_slots[0]; sl < c.probe_slots[1] && sl < T; ++sl) {
    unsigned long long lo[kProbeLaunches], hi[kProbeLaunches];
    for (int k = 0; k < kProbeLaunches; ++k) {
      lo[k] = ~0ull;
      hi[k] = 0;
      const unsigned long long* r = tk.data() + ((size_t)k * T + sl) * kProbeWG * 2;
      for (int w = 0; w < kProbeWG; ++w)
        if (r[2 * w + 1] > r[2 * w] && r[2 * w] != 0) {
          lo[k] = std::min(lo[k], r[2 * w]);
          hi[k] = std::max(hi[k], r[2 * w + 1]);
        }
      if (hi[k] > lo[k]) {
        ms[k] += (double)(hi[k] - lo[k]) / c.wall_khz;
        n[k] += 1;
      }
    }
    // a launch's predecessor is the previous launch of the chain that ran (the fused step has no cross-q launch)
    for (int i = 1, p = chain[0]; i < nchain; ++i) {
      const int k = chain[i];
      if (hi[k] == 0) continue;
      if (hi[p] > 0 && hi[k] > hi[p]) {
        e2e[k] += (double)(hi[k] - hi[p]) / c.wall_khz;
        e2e_n[k] += 1;
      }
      p = k;
    }
  }
  for (int k = 0; k < kProbeLaunches; ++k) {
    if (n[k]) ms[k] /= n[k];
    if (e2e_n[k]) e2e[k] /= e2e_n[k];
  }
}

wmx_status wmx_ctx_probe_stats(wmx_ctx* x, float* avg_ms, int* n, double* bytes) {
  return guard([&] {
    Ctx& c = x->c;
    double ms[kProbeLaunches], e2e[kProbeLaunches];
    int cnt[kProbeLaunches], e2e_n[kProbeLaunches];
    probe_collect(c, ms, cnt, e2e, e2e_n);
    *n = cnt[kProbeCross];
    *avg_ms = (float)ms[kProbeCross];
    *bytes = c.probe_bytes[kProbeCross];
  });
}

wmx_status wmx_ctx_probe_launches(wmx_ctx* x, float* span_ms, double* bytes, int* span_n, float* e2e_ms, int* e2e_n) {
  return guard([&] {
    Ctx& c = x->c;
    double ms[kProbeLaunches], e2e[kProbeLaunches];
    int cnt[kProbeLaunches], en[kProbeLaunches];
    probe_collect(c, ms, cnt, e2e, en);
    for (int k = 0; k < kProbeLaunches; ++k) {
      span_ms[k] = (float)ms[k];
      bytes[k] = c.probe_bytes[k];
      span_n[k] = cnt[k];
      if (e2e_ms) e2e_ms[k] = (float)e2e[k];
      if (e2e_n) e2e_n[k] = en[k];
    }
  });
}

// the lockstep barriers alone, for host tests without a GPU (tests/test_lockstep.py): join group `key` of n members
// (created on first use); op 0 = the start barrier, 1 = a chunk barrier, 2 = leave; *ok = 1 when every member
// expected arrived within timeout_us
wmx_status wmx_debug_lockstep_arrive(int key, int n_members, int op, int timeout_us, int* ok) {
  return guard([&] {
    WMX_CHECK(key != 0 && n_members >= 2 && n_members <= 64 && timeout_us >= 0 && ok && op >= 0 && op <= 2,
              "debug_lockstep: args");
    std::shared_ptr<Lockstep> p;
    {
      std::lock_guard<std::mutex> g(g_lockstep_mu);
      auto& q = g_lockstep[key];
      if (!q) {
        q = std::make_shared<Lockstep>();
        q->n = n_members;
      }
      WMX_CHECK(q->n == n_members, "debug_lockstep: this key was created with another member count");
      p = q;
    }
    if (op == 2) {
      p->leave();
      *ok = 1;
    } else {
      *ok = (op == 0 ? p->arrive(std::chrono::microseconds(timeout_us)) : p->chunk(std::chrono::microseconds(timeout_us)))
                ? 1 : 0;
    }
  });
}

wmx_status wmx_ctx_set_lockstep(wmx_ctx* x, int key, int n_members) {
  return guard([&] {
    Ctx& c = x->c;
    if (key == 0) {
      c.lockstep.reset();
      return;
    }
    WMX_CHECK(n_members >= 2 && n_members <= 64, "lockstep: 2..64 members");
    std::lock_guard<std::mutex> g(g_lockstep_mu);
    auto& p = g_lockstep[key];
    if (!p) {
      p = std::make_shared<Lockstep>();
      p->n = n_members;
    }
    WMX_CHECK(p->n == n_members, "lockstep: this key was created with another member count");
    c.lockstep = p;
  });
}

wmx_status wmx_ctx_probe_ticks(wmx_ctx* x, uint64_t* lo_hi, int* n_steps, double* wall_khz) {
  return guard([&] {
    Ctx& c = x->c;
    WMX_CHECK(n_steps && wall_khz, "probe_ticks: null argument");
    const int T = c.Tctx;
    const int s0 = c.probe_slots[0], s1 = std::min(c.probe_slots[1], T);
    *n_steps = std::max(0, s1 - s0);
    *wall_khz = c.wall_khz;
    if (!lo_hi || *n_steps == 0) return;
    std::vector<unsigned long long> tk((size_t)kProbeLaunches * T * kProbeWG * 2);
    WMX_HIP(hipStreamSynchronize(c.st));
    WMX_HIP(hipMemcpy(tk.data(), c.probe_buf, tk.size() * 8, hipMemcpyDeviceToHost));
    for (int sl = s0; sl < s1; ++sl)
      for (int k = 0; k < kProbeLaunches; ++k) {
        unsigned long long lo = ~0ull, hi = 0;
        const unsigned long long* r = tk.data() + ((size_t)k * T + sl) * kProbeWG * 2;
        for (int w = 0; w < kProbeWG; ++w)
          if (r[2 * w + 1] > r[2 * w] && r[2 * w] != 0) {
            lo = std::min(lo, r[2 * w]);
            hi = std::max(hi, r[2 * w + 1]);
          }
        uint64_t* o = lo_hi + ((size_t)(sl - s0) * kProbeLaunches + k) * 2;
        o[0] = hi > lo ? lo : 0;
        o[1] = hi > lo ? hi : 0;
      }
  });
}

wmx_status wmx_ctx_bench_kernel(wmx_ctx* x, int kernel, int B, int iters, float* avg_ms, double* bytes, double* flops) {
  return guard([&] {
    Ctx& c = x->c;
    Model& m = *c.m;
    WMX_CHECK(B >= 1 && B <= c.maxB && iters >= 1, "bench_kernel: args");
    WMX_HIP(hipSetDevice(m.device));
    const int da = m.d.n_audio_state, dt = m.d.n_text_state, Lt = m.d.n_text_layer, H = m.d.n_text_head;
    const int R = c.K * B;
    double by = 0, fl = 0;
    std::function<void()> fn;
    if (kernel == 0) {
      DecAttnArgs a{};
      a.q = c.dcq;
      a.q_ld = dt;
      a.o = c.dao;
      a.R = R;
      a.Tn = 1;
      a.H = H;
      a.d = dt;
      set_cross_images(c, a, 0);
      a.Tk = 1500;
      a.rows_per_win = c.K;
      const double eb = m.kv8 ? 1.0 : 2.0;  // image / weight bytes per element (fp8 decode: 1)
      by = (double)B * 1500 * 2 * dt * eb + 2.0 * R * dt * 2;
      fl = 4.0 * R * 1500 * dt;
      if (c.xq_fused) {  // the decode step's form: the query projection inside (reads LN2 rows + wcq)
        a.wq = m.kv8 ? reinterpret_cast<const uint16_t*>(m.dec[0].q8cq) : m.dec[0].wcq;
        a.wq_scale = m.kv8 ? m.dec[0].s8cq : nullptr;
        a.qin = c.dhb;
        a.qin_ld = dt;
        a.qbias = m.dec[0].bcq;
        by += (double)dt * dt * eb;
        fl += 2.0 * R * dt * dt;
      }
      a.xcnt = c.xa_cnt;
      fn = [&c, a] { launch_cross_attn(c.dt, a, c.xa_ws, c.st); };
    } else if (kernel == 1) {
      const long rows = (long)B * 1500;
      by = (double)rows * da * 2 + 4.0 * da * da * 2 + (double)rows * 4 * da * 2;
      fl = 2.0 * rows * 4 * da * da;
      fn = [&c, &m, rows, da] {
        gemm(c, c.ehb, da, m.enc[0].wfc1, da, (int)rows, 4 * da, da, epi(EPI_GELU16, m.enc[0].bfc1, c.ef1, 4 * da));
      };
    } else if (kernel == 2) {
      AttnArgs a{};
      a.q = c.eqkv;
      a.k = c.eqkv + da;
      a.v = c.eqkv + 2 * da;
      a.q_ld = a.k_ld = a.v_ld = 3 * da;
      a.q_bstride = a.k_bstride = a.v_bstride = 1500L * 3 * da;
      a.o = c.eao;
      a.o_ld = da;
      a.o_bstride = 1500L * da;
      a.B = B;
      a.H = m.d.n_audio_head;
      a.Tq = a.Tk = 1500;
      a.head_stride = 64;
      by = (double)B * 1500 * 4 * da * 2;
      fl = 4.0 * B * m.d.n_audio_head * 1500.0 * 1500.0 * 64;
      fn = [&c, a] { launch_attn_encoder(c.dt, a, c.st); };
    } else if (kernel == 3) {
      std::vector<long> lens(B, std::min<long>(480000, c.max_samples));
      WMX_HIP(hipMemcpy(c.lens, lens.data(), B * sizeof(long), hipMemcpyHostToDevice));
      WMX_HIP(hipMemset(c.seek, 0, B * 4));
      by = (double)B * (480000.0 * 4 + m.d.n_mels * 3000.0 * 4);
      fl = (double)B * 3001 * logmel_flops_per_frame();
      fn = [&c, &m, B] {
        launch_logmel(c.pcm, std::min<long>(480000, c.max_samples), c.lens, c.seek, B, 3001, m.mel_first, m.mel_count,
                      m.mel_off, m.mel_w, m.d.n_mels, c.mel_stats, c.mel_stats_cap, c.mel, c.st);
      };
    } else if (kernel == 4) {
      by = 4.0 * dt * dt * (m.w8 ? 1 : 2) + (double)R * dt * 2 + (double)R * 4 * dt * 2;
      fl = 2.0 * R * 4 * dt * dt;
      fn = [&c, &m, R, dt] {
        gemm_p(c, c.dhb, dt, m.dec[0].wfc1, R, 4 * dt, dt, epi(EPI_GELU16, m.dec[0].bfc1, c.df1, 4 * dt), nullptr,
               w8_of(m, m.dec[0].q8fc1, m.dec[0].s8fc1));
      };
    } else if (kernel == 5) {
      DecAttnArgs a{};
      a.q = c.dq;
      a.q_ld = dt;
      a.o = c.dao;
      a.R = R;
      a.Tn = 1;
      a.H = H;
      a.d = dt;
      a.kc = c.kc;
      a.vc = c.vc;
      a.kv_R = c.R;
      a.anc = c.beam ? c.anc : nullptr;
      a.anc_ld = c.Tctx;
      a.pad = c.pad_row;
      a.slot0 = c.slot;
      int s = 0;
      WMX_HIP(hipMemcpy(&s, c.slot, 4, hipMemcpyDeviceToHost));
      by = (double)R * (s + 1) * dt * 2 * 2;
      fl = 4.0 * R * (s + 1) * dt;
      fn = [&c, a] { launch_self_attn(c.dt, a, c.st); };
    } else if (kernel == 11) {
      // decoder fc1 of the mixed step: LN3 folded into the weights, the row statistics merged in the epilogue
      WMX_CHECK(m.mixed, "bench_kernel: the LayerNorm-folded fc1 exists on mixed-step models only");
      by = 4.0 * dt * dt * 2 + (double)R * dt * 2 + (double)R * 4 * dt * 2;
      fl = 2.0 * R * 4 * dt * dt;
      fn = [&c, &m, R, dt] {
        Epi e1 = epi(EPI_LNFOLD_GELU16, nullptr, c.df1, 4 * dt);
        e1.c1 = m.dec[0].c1fc1;
        e1.c2 = m.dec[0].c2fc1;
        e1.stats = c.rstat;
        e1.stats_ld = dt / 16;
        gemm_p(c, c.dhb, dt, m.dec[0].ffc1, R, 4 * dt, dt, e1);
      };
    } else if (kernel == 6) {
      // the whole encoder (conv front end + every layer + final LN) over B windows: its MFMA work per window
      const double T = 1500, M = m.d.n_mels, Ha = m.d.n_audio_head, La = m.d.n_audio_layer;
      fl = B * (2.0 * 3000 * 3 * M * da + 2.0 * T * 3 * da * da +
                La * (2.0 * T * da * 3 * da + 4.0 * Ha * T * T * 64 + 2.0 * T * da * da + 4.0 * T * da * 4 * da));
      by = (double)La * 12 * da * da * 2;
      fn = [&c, B] { encode(c, B); };
    } else if (kernel >= 7 && kernel <= 9) {
      // decode-step projections on packed weights, split-K partial launches: 7 qkv, 8 a d x d projection, 9 fc2
      const int N = kernel == 7 ? 3 * dt : dt, K = kernel == 9 ? 4 * dt : dt;
      const uint16_t* W = kernel == 7 ? m.dec[0].wqkv : kernel == 8 ? m.dec[0].wo : m.dec[0].wfc2;
      const DecLayer& L0 = m.dec[0];
      const W8 w8 = kernel == 7 ? w8_of(m, L0.q8qkv, L0.s8qkv) : kernel == 8 ? w8_of(m, L0.q8o, L0.s8o)
                                                                             : w8_of(m, L0.q8fc2, L0.s8fc2);
      const uint16_t* A = kernel == 9 ? c.df1 : c.dhb;
      by = (double)N * K * (m.w8 ? 1 : 2) + (double)R * K * 2 + (double)R * N * 2;
      fl = 2.0 * R * N * K;
      fn = [&c, A, W, R, N, K, w8] { gemm_p_part(c, A, K, W, R, N, K, w8); };
    } else if (kernel == 10) {
      // reduce_ln after a d x d projection: x += bias + sum of its split-K partials; LN(x) -> 16-bit
      const int S = packed_splits(R, dt, dt, c.part_elems);
      const int S2 = S == 1 ? 2 : S;
      by = (double)S2 * R * dt * 4 + 2.0 * R * dt * 4 + (double)R * dt * 2;
      fl = 0;
      fn = [&c, &m, S2, R, dt] {
        launch_reduce_ln(c.dt, c.part, S2, m.dec[0].bo, c.dx, m.dec[0].ln2g, m.dec[0].ln2b, c.dhb, R, dt, c.st);
      };
    } else {
      WMX_CHECK(false, "bench_kernel: unknown kernel");
    }
    fn();  // warm
    WMX_HIP(hipEventRecord(c.ev[0], c.st));
    for (int i = 0; i < iters; ++i) fn();
    WMX_HIP(hipEventRecord(c.ev[1], c.st));
    WMX_HIP(hipEventSynchronize(c.ev[1]));
    float ms = 0;
    WMX_HIP(hipEventElapsedTime(&ms, c.ev[0], c.ev[1]));
    *avg_ms = ms / iters;
    *bytes = by;
    *flops = fl;
  });
}

}  // extern "C"

// ---- Silero VAD (wmx_vad.hip) ----
struct wmx_vad {
  int device = 0, max_streams = 0, max_windows = 0;
  hipStream_t st = nullptr;
  char* base = nullptr;  // one allocation: weights, state, context, pcm staging, encoder outputs, probs, slots
  float *W = nullptr, *state = nullptr, *ctx = nullptr, *pcm = nullptr, *enc = nullptr, *probs = nullptr;
  int* slots = nullptr;
  unsigned loaded = 0;  // bit per tensor of vad_tensors()
};

namespace {
struct VadTensor {
  const char* name;
  long n, off;
  int transpose_rows;  // > 0: [rows][n / rows] stored transposed
};
const std::vector<VadTensor>& vad_tensors() {
  static const std::vector<VadTensor> t = {
      {"stft.forward_basis_buffer", 258L * 256, kVadOffBasis, 0},
      {"encoder.0.reparam_conv.weight", 128L * 129 * 3, kVadOffC0w, 0},
      {"encoder.0.reparam_conv.bias", 128, kVadOffC0b, 0},
      {"encoder.1.reparam_conv.weight", 64L * 128 * 3, kVadOffC1w, 0},
      {"encoder.1.reparam_conv.bias", 64, kVadOffC1b, 0},
      {"encoder.2.reparam_conv.weight", 64L * 64 * 3, kVadOffC2w, 0},
      {"encoder.2.reparam_conv.bias", 64, kVadOffC2b, 0},
      {"encoder.3.reparam_conv.weight", 128L * 64 * 3, kVadOffC3w, 0},
      {"encoder.3.reparam_conv.bias", 128, kVadOffC3b, 0},
      {"decoder.rnn.weight_ih", 512L * 128, kVadOffWihT, 512},
      {"decoder.rnn.weight_hh", 512L * 128, kVadOffWhhT, 512},
      {"decoder.rnn.bias_ih", 512, kVadOffBih, 0},
      {"decoder.rnn.bias_hh", 512, kVadOffBhh, 0},
      {"decoder.decoder.2.weight", 128, kVadOffW2, 0},
      {"decoder.decoder.2.bias", 1, kVadOffB2, 0},
  };
  return t;
}

void vad_check_call(wmx_vad* v, int64_t stride, const int32_t* slots, int S, int nwin) {
  WMX_CHECK(v && slots, "null argument");
  WMX_CHECK(v->loaded == (1u << vad_tensors().size()) - 1, "vad: weights not fully loaded (wmx_vad_set_tensor)");
  WMX_CHECK(S >= 1 && S <= v->max_streams, "vad: stream count out of range");
  WMX_CHECK(nwin >= 1 && nwin <= v->max_windows, "vad: window count out of range");
  WMX_CHECK(stride >= (int64_t)nwin * kVadWindow, "vad: stride shorter than nwin * 512 samples");
  std::vector<char> seen(v->max_streams, 0);
  for (int i = 0; i < S; ++i) {
    WMX_CHECK(slots[i] >= 0 && slots[i] < v->max_streams, "vad: slot out of range");
    WMX_CHECK(!seen[slots[i]], "vad: a slot appears twice in one call");
    seen[slots[i]] = 1;
  }
}
}  // namespace

extern "C" {

wmx_status wmx_vad_create(int device, int max_streams, int max_windows, wmx_vad** out) {
  return guard([&] {
    WMX_CHECK(out && max_streams >= 1 && max_windows >= 1 && max_streams <= 65536 && max_windows <= 4096,
              "vad: bad sizes");
    auto* v = new wmx_vad();
    try {
      v->device = device;
      v->max_streams = max_streams;
      v->max_windows = max_windows;
      WMX_HIP(hipSetDevice(device));
      WMX_HIP(hipStreamCreateWithFlags(&v->st, hipStreamNonBlocking));
      const size_t MS = max_streams, MW = max_windows;
      const size_t nW = (kVadWeights + 63) / 64 * 64, nS = MS * 2 * kVadHidden, nC = MS * kVadContext,
                   nP = MS * MW * kVadWindow, nE = MS * MW * kVadHidden, nPr = MS * MW;
      const size_t floats = nW + nS + nC + nP + nE + (nPr + 63) / 64 * 64;
      WMX_HIP(hipMalloc(&v->base, floats * 4 + MS * 4));
      WMX_HIP(hipMemset(v->base, 0, floats * 4 + MS * 4));
      float* f = (float*)v->base;
      v->W = f;
      v->state = f + nW;
      v->ctx = v->state + nS;
      v->pcm = v->ctx + nC;
      v->enc = v->pcm + nP;
      v->probs = v->enc + nE;
      v->slots = (int*)(f + floats);
    } catch (...) {
      if (v->base) (void)hipFree(v->base);
      if (v->st) (void)hipStreamDestroy(v->st);
      delete v;
      throw;
    }
    *out = v;
  });
}

void wmx_vad_free(wmx_vad* v) {
  if (!v) return;
  (void)hipSetDevice(v->device);
  if (v->base) (void)hipFree(v->base);
  if (v->st) (void)hipStreamDestroy(v->st);
  delete v;
}

void* wmx_vad_stream(wmx_vad* v) { return v ? (void*)v->st : nullptr; }

wmx_status wmx_vad_set_tensor(wmx_vad* v, const char* name, const float* data, int64_t n) {
  return guard([&] {
    WMX_CHECK(v && name && data, "null argument");
    const auto& ts = vad_tensors();
    for (size_t i = 0; i < ts.size(); ++i) {
      if (std::string(name) != ts[i].name) continue;
      WMX_CHECK(n == ts[i].n, std::string("vad: size mismatch for ") + name);
      std::vector<float> img(data, data + n);
      if (ts[i].transpose_rows > 0) {  // [rows][cols] -> [cols][rows]
        const long rows = ts[i].transpose_rows, cols = n / rows;
        for (long r = 0; r < rows; ++r)
          for (long c = 0; c < cols; ++c) img[c * rows + r] = data[r * cols + c];
      }
      WMX_HIP(hipSetDevice(v->device));
      WMX_HIP(hipMemcpy(v->W + ts[i].off, img.data(), n * 4, hipMemcpyHostToDevice));
      v->loaded |= 1u << i;
      return;
    }
    WMX_CHECK(false, std::string("vad: unknown tensor ") + name);
  });
}

wmx_status wmx_vad_reset(wmx_vad* v, int slot) {
  return guard([&] {
    WMX_CHECK(v && slot < v->max_streams, "vad: slot out of range");
    WMX_HIP(hipSetDevice(v->device));
    if (slot < 0) {
      WMX_HIP(hipMemsetAsync(v->state, 0, (size_t)v->max_streams * 2 * kVadHidden * 4, v->st));
      WMX_HIP(hipMemsetAsync(v->ctx, 0, (size_t)v->max_streams * kVadContext * 4, v->st));
    } else {
      WMX_HIP(hipMemsetAsync(v->state + (size_t)slot * 2 * kVadHidden, 0, 2 * kVadHidden * 4, v->st));
      WMX_HIP(hipMemsetAsync(v->ctx + (size_t)slot * kVadContext, 0, kVadContext * 4, v->st));
    }
    WMX_HIP(hipStreamSynchronize(v->st));
  });
}

wmx_status wmx_vad_process_device(wmx_vad* v, const float* pcm_dev, int64_t stride, const int32_t* slots, int S,
                                  int nwin, float* probs_dev) {
  return guard([&] {
    vad_check_call(v, stride, slots, S, nwin);
    WMX_CHECK(pcm_dev && probs_dev, "null argument");
    WMX_HIP(hipSetDevice(v->device));
    // the slot table is rewritten below: an earlier call's launches on this stream must have read it
    WMX_HIP(hipStreamSynchronize(v->st));
    WMX_HIP(hipMemcpyAsync(v->slots, slots, (size_t)S * 4, hipMemcpyHostToDevice, v->st));
    launch_vad(v->W, pcm_dev, (long)stride, v->ctx, v->state, v->slots, S, nwin, v->enc, probs_dev, v->st);
  });
}

wmx_status wmx_vad_process(wmx_vad* v, const float* pcm, int64_t stride, const int32_t* slots, int S, int nwin,
                           float* probs) {
  return guard([&] {
    vad_check_call(v, stride, slots, S, nwin);
    WMX_CHECK(pcm && probs, "null argument");
    WMX_HIP(hipSetDevice(v->device));
    const long row = (long)nwin * kVadWindow;
    WMX_HIP(hipMemcpy2DAsync(v->pcm, row * 4, pcm, (size_t)stride * 4, row * 4, S, hipMemcpyHostToDevice, v->st));
    WMX_HIP(hipMemcpyAsync(v->slots, slots, (size_t)S * 4, hipMemcpyHostToDevice, v->st));
    launch_vad(v->W, v->pcm, row, v->ctx, v->state, v->slots, S, nwin, v->enc, v->probs, v->st);
    WMX_HIP(hipMemcpyAsync(probs, v->probs, (size_t)S * nwin * 4, hipMemcpyDeviceToHost, v->st));
    WMX_HIP(hipStreamSynchronize(v->st));
  });
}

}  // extern "C"
