// Decode-loop kernels: logit rules, log-softmax, greedy argmax / beam top-k and
// beam bookkeeping, language detection, no-speech probability, alignment-matrix post-processing.
//
// Rules restated from openai-whisper decoding.py (CTranslate2 re-implements the same): SuppressBlank (step 0:
// " " and <|endoftext|>), SuppressTokens (bitmask), ApplyTimestampRules (no <|notimestamps|>, timestamps in pairs,
// monotonic, initial timestamp <= max_initial_timestamp_index, force a timestamp when
// logsumexp(timestamps) > max(text)).  The masks are evaluated on the fly from a 5-int per-row state, so the
// logits are read once for statistics and once for the argmax / top-k (never rewritten).
// Beam search: openai BeamSearchDecoder with patience; candidates ranked by (score desc, beam asc, token asc).
// Beams are reordered by copying token history + ancestry rows (ints), never the KV cache.
#include "wmx_common.h"
#include "wmx_decode.h"

namespace wmx {

struct RowState {  // SoA pointers, one entry per row
  int* ns;         // sampled tokens so far
  int* last;
  int* pen;
  int* last_ts;    // last timestamp token or -1
  int* done;
  float* sum_lp;
};

// every rule except the suppress bitmask (the caller tests that word)
__device__ inline bool allowed_rules(const RuleOpts& o, int t, int ns, bool last_ts, bool pen_ts, int lts) {
  if (t == o.no_ts) return false;
  if (o.suppress_blank && ns == 0 && (t == o.blank || t == o.eot)) return false;
  if (!o.without_ts) {
    if (last_ts) {
      if (pen_ts) {
        if (t >= o.tb) return false;
      } else if (t < o.eot) {
        return false;
      }
    }
    if (lts >= 0) {
      const int ts_last = (last_ts && !pen_ts) ? lts : lts + 1;
      if (t >= o.tb && t < ts_last) return false;
    }
    if (ns == 0) {
      if (t < o.tb) return false;
      if (o.max_init >= 0 && t > o.tb + o.max_init) return false;
    }
  }
  return true;
}

__device__ inline bool allowed(const RuleOpts& o, int t, int ns, bool last_ts, bool pen_ts, int lts) {
  if ((o.mask[t >> 5] >> (t & 31)) & 1u) return false;
  return allowed_rules(o, t, ns, last_ts, pen_ts, lts);
}

struct MS {  // online max/sum
  float m, s;
};
__device__ inline MS ms_add(MS a, float v) {
  if (v == -INFINITY) return a;
  if (v > a.m) {
    a.s = a.s * __expf(a.m - v) + 1.f;
    a.m = v;
  } else {
    a.s += __expf(v - a.m);
  }
  return a;
}
// branch-free ms_add: identical values (the skipped factor is exp(0) = 1 and s * 1 is exact)
__device__ inline MS ms_add_nb(MS a, float v) {
  const float m = fmaxf(a.m, v);
  const float s = a.s * __expf(a.m - m) + __expf(v - m);
  return v == -INFINITY ? a : MS{m, s};
}
__device__ inline MS ms_merge(MS a, MS b) {
  if (b.m == -INFINITY) return a;
  if (a.m == -INFINITY) return b;
  const float m = fmaxf(a.m, b.m);
  return MS{m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}
__device__ inline float ms_lse(MS a) { return a.m == -INFINITY ? -INFINITY : a.m + __logf(a.s); }
// wave-wide ms_merge on DPP / permlane exchanges (all lanes active; ms_merge is commutative, so every lane ends
// with the same pair)
template <int CTRL>
__device__ inline MS ms_step_dpp(MS a) {
  return ms_merge(a, MS{dpp_mov<CTRL>(a.m), dpp_mov<CTRL>(a.s)});
}
__device__ inline MS wave_ms(MS a) {
  a = ms_step_dpp<kDppXor1>(a);
  a = ms_step_dpp<kDppXor2>(a);
  a = ms_step_dpp<kDppHalfMirror>(a);
  a = ms_step_dpp<kDppMirror>(a);
  {
    const auto m = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.m), __float_as_uint(a.m), false, false);
    const auto sv = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.s), __float_as_uint(a.s), false, false);
    a = ms_merge(MS{__uint_as_float(m[0]), __uint_as_float(sv[0])}, MS{__uint_as_float(m[1]), __uint_as_float(sv[1])});
  }
  {
    const auto m = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.m), __float_as_uint(a.m), false, false);
    const auto sv = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.s), __float_as_uint(a.s), false, false);
    a = ms_merge(MS{__uint_as_float(m[0]), __uint_as_float(sv[0])}, MS{__uint_as_float(m[1]), __uint_as_float(sv[1])});
  }
  return a;
}

constexpr int kSelThreads = 512;
constexpr int kMaxKP = 9;

// better(a, b): value desc, index asc
__device__ inline bool better(float va, int ia, float vb, int ib) { return va > vb || (va == vb && ia < ib); }

// ---- phase A: one block per (row, vocab slice): masked statistics + top-KP of allowed text and timestamp
//      tokens, kept separately because whether text is masked depends on the whole row ----
constexpr int kSlices = 16, kSelA = 256;
constexpr int kSelPer = 3584;                   // vocab entries per slice (16 x 3584 >= 51866), a multiple of 2 kSelA
constexpr int kSelNL = kSelPer / (2 * kSelA);   // 8-byte loads per thread per slice

struct TopK {
  float v[kMaxKP];
  int i[kMaxKP];
};

__device__ inline void topk_init(TopK& t) {
#pragma unroll
  for (int k = 0; k < kMaxKP; ++k) {
    t.v[k] = -INFINITY;
    t.i[k] = 0x7FFFFFFF;
  }
}
// sorted insert with compile-time indices only (runtime-indexed register arrays would spill to scratch)
__device__ inline void topk_push(TopK& t, float v, int i, int KP) {
#pragma unroll
  for (int k = 0; k < kMaxKP; ++k) {
    if (k < KP && better(v, i, t.v[k], t.i[k])) {
      const float tv = t.v[k];
      const int ti = t.i[k];
      t.v[k] = v;
      t.i[k] = i;
      v = tv;
      i = ti;
    }
  }
}
// compile-time list length, branch-free compare-and-swap chain (the runtime-KP form above compiles to an
// exec-mask branch per slot; this is ~6 VALU per slot).  better_nb: better() without short-circuit branches.
__device__ inline bool better_nb(float va, int ia, float vb, int ib) { return (va > vb) | ((va == vb) & (ia < ib)); }
template <int KPT>
__device__ inline void topk_push_c(TopK& t, float v, int i) {
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const bool sw = better_nb(v, i, t.v[k], t.i[k]);
    const float tv = t.v[k];
    const int ti = t.i[k];
    t.v[k] = sw ? v : tv;
    t.i[k] = sw ? i : ti;
    v = sw ? tv : v;
    i = sw ? ti : i;
  }
}
__device__ inline void topk_pop(TopK& t) {
#pragma unroll
  for (int k = 0; k + 1 < kMaxKP; ++k) {
    t.v[k] = t.v[k + 1];
    t.i[k] = t.i[k + 1];
  }
  t.v[kMaxKP - 1] = -INFINITY;
  t.i[kMaxKP - 1] = 0x7FFFFFFF;
}

// (v, i) of the best lane of the wave under better(); every lane ends with the same pair.  DPP / permlane
// exchanges (all lanes active): each step keeps the better of this lane's pair and its partner's, and better()
// is a strict total order, so both partners keep the same pair.
template <int CTRL>
__device__ inline void argmax_step_dpp(float& v, int& i) {
  const float v2 = dpp_mov<CTRL>(v);
  const int i2 = __builtin_amdgcn_mov_dpp(i, CTRL, 0xF, 0xF, false);
  if (better(v2, i2, v, i)) {
    v = v2;
    i = i2;
  }
}
__device__ inline void argmax_pick(float& v, int& i, const uint32_t* rv, const uint32_t* ri) {
  // rv / ri: a permlane swap of (v, v) and (i, i): elements 0 come from one lane, elements 1 from the other
  const float va = __uint_as_float(rv[0]), vb = __uint_as_float(rv[1]);
  const int ia = (int)ri[0], ib = (int)ri[1];
  if (better(va, ia, vb, ib)) {
    v = va;
    i = ia;
  } else {
    v = vb;
    i = ib;
  }
}
__device__ inline void wave_argmax(float& v, int& i) {
  argmax_step_dpp<kDppXor1>(v, i);
  argmax_step_dpp<kDppXor2>(v, i);
  argmax_step_dpp<kDppHalfMirror>(v, i);
  argmax_step_dpp<kDppMirror>(v, i);
  {
    const auto rv = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto ri = __builtin_amdgcn_permlane16_swap((uint32_t)i, (uint32_t)i, false, false);
    const uint32_t a[2] = {rv[0], rv[1]}, b[2] = {ri[0], ri[1]};
    argmax_pick(v, i, a, b);
  }
  {
    const auto rv = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const auto ri = __builtin_amdgcn_permlane32_swap((uint32_t)i, (uint32_t)i, false, false);
    const uint32_t a[2] = {rv[0], rv[1]}, b[2] = {ri[0], ri[1]};
    argmax_pick(v, i, a, b);
  }
}

// block-wide: extract the KP best heads of all threads' lists into ov / oi (rank order; (-inf, INT_MAX) pads).
// Each wave first extracts its own KP best (KP wave arg-maxes, the owning lane pops its head: indices are
// unique, so exactly one lane owns the pair), then wave 0 extracts the KP best of the waves' candidates.
// Every thread of the block must call it.  rv / ri: scratch of at least (NT / 64) * kMaxKP entries.
template <int NT>
__device__ inline void block_topk(TopK& t, int KP, float* ov, int* oi, float* rv, int* ri) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int k = 0; k < KP; ++k) {
    float v = t.v[0];
    int i = t.i[0];
    wave_argmax(v, i);
    if (t.i[0] == i && i != 0x7FFFFFFF) topk_pop(t);
    if (NW == 1) {
      if (lane == 0) {
        ov[k] = v;
        oi[k] = i;
      }
    } else if (lane == 0) {
      rv[wave * kMaxKP + k] = v;
      ri[wave * kMaxKP + k] = i;
    }
  }
  if (NW == 1) return;
  __syncthreads();
  if (wave == 0) {
    float cv = -INFINITY;
    int ci = 0x7FFFFFFF;
    if (lane < NW * KP) {
      cv = rv[(lane / KP) * kMaxKP + lane % KP];
      ci = ri[(lane / KP) * kMaxKP + lane % KP];
    }
    for (int k = 0; k < KP; ++k) {
      float v = cv;
      int i = ci;
      wave_argmax(v, i);
      if (ci == i && i != 0x7FFFFFFF) {
        cv = -INFINITY;
        ci = 0x7FFFFFFF;
      }
      if (lane == 0) {
        ov[k] = v;
        oi[k] = i;
      }
    }
  }
}

// sampling noise: splitmix64 of the counter ((row * 1024 + slot) * 65536 + token) offset by seed * golden ratio;
// u = (top 23 bits * 2 + 1) / 2^25 in (0, 1), exact in f32; Gumbel = -log(-log(u)).  Restated bit for bit by
// oracle/whisper_np.py::sample_gumbel (the replay test).
__device__ inline float sample_gumbel(uint32_t seed, int row, int slot, int tok) {
  uint64_t z = ((uint64_t)row * 1024u + (uint64_t)slot) * 65536u + (uint64_t)tok + (uint64_t)seed * 0x9E3779B97F4A7C15ull;
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)((uint32_t)(z >> 41) * 2u + 1u) * 2.98023223876953125e-8f;  // 2^-25
  return -logf(-logf(u));
}

// workspace per (row, slice): [0..4] stats (text.m, text.s, ts.m, ts.s, text max), then KP text (v,i), KP ts (v,i)
__device__ inline int sel_ws_stride(int KP) { return 5 + 4 * KP; }

// SAMPLE: the top-KP lists rank tokens by the sampling key logit / T + Gumbel noise (KP = 1: the Gumbel-max sample);
// the statistics stay on the raw logits (log-probabilities and the timestamp rule, as openai / CT2 compute them)
template <int KP, bool SAMPLE = false>
__global__ __launch_bounds__(kSelA) void logits_select_a(const float* __restrict__ logits, int ldl, RuleOpts o,
                                                         RowState rs, const int* row_map, float* __restrict__ ws) {
  const int r = blockIdx.x, sl = blockIdx.y;
  const int sample_slot = SAMPLE ? *o.slot : 0;
  const uint32_t sample_seed = SAMPLE ? *o.seed : 0u;
  const int lrow = row_map ? row_map[r] : r;
  const float* x = logits + (long)lrow * ldl;
  const int ns = rs.ns[r], lt = rs.last[r], pt = rs.pen[r], lts = rs.last_ts[r];
  const bool last_ts = ns >= 1 && lt >= o.tb;
  const bool pen_ts = ns < 2 || pt >= o.tb;
  const int tid = threadIdx.x;
  MS text{-INFINITY, 0.f}, ts{-INFINITY, 0.f};
  float tmax = -INFINITY;
  TopK ktx, kts;
  topk_init(ktx);
  topk_init(kts);
  // the slice's values (pairs t, t+1 per 8-byte load) and suppress-mask words, all loaded before any use
  const int t0 = sl * kSelPer;
  float2 xv[kSelNL];
  unsigned mw[kSelNL];
#pragma unroll
  for (int u = 0; u < kSelNL; ++u) {
    const int t = t0 + 2 * (tid + u * kSelA);
    xv[u] = t + 1 < o.V ? *reinterpret_cast<const float2*>(x + t)
                        : make_float2(t < o.V ? x[min(t, o.V - 1)] : -INFINITY, -INFINITY);
    mw[u] = t < o.V ? o.mask[t >> 5] : 0u;
  }
#pragma unroll
  for (int u = 0; u < kSelNL; ++u) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int t = t0 + 2 * (tid + u * kSelA) + hh;
      // a suppressed token enters as (-inf, INT_MAX): a no-op for the statistics and the top-KP lists
      const bool ok = t < o.V && !((mw[u] >> (t & 31)) & 1u) && allowed_rules(o, t, ns, last_ts, pen_ts, lts);
      const float v = ok ? (hh ? xv[u].y : xv[u].x) : -INFINITY;
      const int ti = ok ? t : 0x7FFFFFFF;
      const float key = SAMPLE ? (ok ? v * o.inv_temp + sample_gumbel(sample_seed, r, sample_slot, t) : -INFINITY) : v;
      if (t < o.tb) {  // wave-uniform except in the slice that holds timestamp_begin
        text = ms_add_nb(text, v);
        tmax = fmaxf(tmax, v);
        topk_push_c<KP>(ktx, key, ti);
      } else {
        ts = ms_add_nb(ts, v);
        topk_push_c<KP>(kts, key, ti);
      }
    }
  }
  text = wave_ms(text);
  ts = wave_ms(ts);
  tmax = wave_max(tmax);
  __shared__ float sm[5][kSelA / 64];
  __shared__ float rv[(kSelA / 64) * kMaxKP];
  __shared__ int ri[(kSelA / 64) * kMaxKP];
  const int wave = tid >> 6, lane = tid & 63;
  if (lane == 0) {
    sm[0][wave] = text.m;
    sm[1][wave] = text.s;
    sm[2][wave] = ts.m;
    sm[3][wave] = ts.s;
    sm[4][wave] = tmax;
  }
  __syncthreads();
  float* w = ws + ((long)r * kSlices + sl) * sel_ws_stride(KP);
  if (tid == 0) {
    MS T{-INFINITY, 0.f}, S{-INFINITY, 0.f};
    float mx = -INFINITY;
    for (int q = 0; q < kSelA / 64; ++q) {
      T = ms_merge(T, MS{sm[0][q], sm[1][q]});
      S = ms_merge(S, MS{sm[2][q], sm[3][q]});
      mx = fmaxf(mx, sm[4][q]);
    }
    w[0] = T.m;
    w[1] = T.s;
    w[2] = S.m;
    w[3] = S.s;
    w[4] = mx;
  }
  __shared__ float ov[kMaxKP];
  __shared__ int oi[kMaxKP];
  block_topk<kSelA>(ktx, KP, ov, oi, rv, ri);
  __syncthreads();
  if (tid < KP) {
    w[5 + tid] = ov[tid];
    w[5 + KP + tid] = __int_as_float(oi[tid]);
  }
  __syncthreads();
  block_topk<kSelA>(kts, KP, ov, oi, rv, ri);
  __syncthreads();
  if (tid < KP) {
    w[5 + 2 * KP + tid] = ov[tid];
    w[5 + 3 * KP + tid] = __int_as_float(oi[tid]);
  }
}

// ---- phase B: one wave per row merges the slices: timestamp-forcing rule, log-softmax normaliser, top-KP ----
template <int KP, bool SAMPLE = false>
__global__ __launch_bounds__(64) void logits_select_b(const float* __restrict__ ws, RuleOpts o,
                                                      int* __restrict__ out_tok, float* __restrict__ out_lp,
                                                      const float* __restrict__ logits, int ldl,
                                                      const int* __restrict__ row_map) {
  static_assert(kSlices <= 64, "one lane per slice");
  const int r = blockIdx.x;
  const int lane = threadIdx.x;
  const float* w = ws + (long)r * kSlices * sel_ws_stride(KP);
  // lane q < kSlices loads slice q's statistics; one wave-wide merge
  MS T{-INFINITY, 0.f}, S{-INFINITY, 0.f};
  float tmax = -INFINITY;
  if (lane < kSlices) {
    const float* x = w + lane * sel_ws_stride(KP);
    T = MS{x[0], x[1]};
    S = MS{x[2], x[3]};
    tmax = x[4];
  }
  T = wave_ms(T);
  S = wave_ms(S);
  tmax = wave_max(tmax);
  const float lse_ts = ms_lse(S);
  const bool mask_text = !o.without_ts && (lse_ts > tmax);
  const float lse_text = ms_lse(T);
  float lse_all;
  if (mask_text) {
    lse_all = lse_ts;
  } else {
    const float m = fmaxf(lse_text, lse_ts);
    lse_all = m == -INFINITY ? -INFINITY : m + __logf(__expf(lse_text - m) + __expf(lse_ts - m));
  }
  // candidates: lane owns up to 3 (slice, kind, k) entries of the 2 * kSlices * KP list
  TopK t;
  topk_init(t);
  const int ncand = 2 * kSlices * KP;
  for (int c = lane; c < ncand; c += 64) {
    const int q = c / (2 * KP), rem = c % (2 * KP), kind = rem / KP, k = rem % KP;
    if (kind == 0 && mask_text) continue;
    const float* x = w + q * sel_ws_stride(KP) + 5 + 2 * KP * kind;
    topk_push_c<KP>(t, x[k], __float_as_int(x[KP + k]));
  }
  __shared__ float rv[1];
  __shared__ int ri[1];
  __shared__ float ov[kMaxKP];
  __shared__ int oi[kMaxKP];
  block_topk<64>(t, KP, ov, oi, rv, ri);
  __syncthreads();
  if (lane < KP) {
    const int bi = oi[lane];
    const float bv = ov[lane];
    // no candidate (every key -inf or NaN: the list keeps its (-inf, INT_MAX) init) -> EOT; any id outside the
    // vocabulary likewise, so a non-finite row can end a hypothesis but never reach the embedding gather
    const bool none = bi < 0 || bi >= o.V;
    out_tok[r * KP + lane] = none ? o.eot : bi;
    if (lane == 0 && o.err && (none || !(fabsf(lse_all) < INFINITY)))
      atomicCAS(o.err, 0, 1 + r + 1024 * (o.err_slot ? *o.err_slot : 0));
    if (SAMPLE) {  // bv is the sampling key: the log-probability comes from the raw logit of the drawn token
      const int lrow = row_map ? row_map[r] : r;
      out_lp[r * KP + lane] = none ? -INFINITY : logits[(long)lrow * ldl + bi] - lse_all;
    } else {
      out_lp[r * KP + lane] = bv == -INFINITY ? -INFINITY : bv - lse_all;
    }
  }
}

// greedy: single block of R threads; appends the token at slot+1, then advances the slot
__global__ void greedy_update_kernel(RowState rs, const int* __restrict__ tok, const float* __restrict__ lp, int R, int tb,
                                     int eot, int* __restrict__ hist, int hist_ld, int* __restrict__ slot,
                                     int* __restrict__ n_done) {
  const int r = threadIdx.x;
  const int s = *slot;
  if (r < R && !rs.done[r]) {
    const int t = tok[r];
    rs.sum_lp[r] += lp[r];
    if (t == eot) {
      rs.done[r] = 1;
      atomicAdd(n_done, 1);
    } else {
      hist[(long)r * hist_ld + s + 1] = t;
      rs.pen[r] = rs.last[r];
      rs.last[r] = t;
      rs.ns[r] += 1;
      if (t >= tb) rs.last_ts[r] = t;
    }
  }
  __syncthreads();
  if (r == 0) *slot = s + 1;
}

// beam: one wave per window ranks K*(K+1) candidates (or K+1 at the first step: all beams identical)
__global__ void beam_select_kernel(RowState rs, const int* __restrict__ ctok, const float* __restrict__ clp, int K,
                                   int max_cand, int eot, const int* __restrict__ slot, const int* __restrict__ hist,
                                   int hist_ld, BeamState bs, int* __restrict__ n_done) {
  const int w = blockIdx.x;
  const int lane = threadIdx.x;
  if (bs.win_done[w]) {
    if (lane == 0) bs.win_active[w] = 0;
    return;
  }
  const int KP = K + 1;
  const int r0 = w * K;
  const bool first = rs.ns[r0] == 0;
  const int nc = first ? KP : K * KP;
  __shared__ float cv[kMaxKP * 8];
  __shared__ int cb[kMaxKP * 8], ct[kMaxKP * 8];
  __shared__ int order[kMaxKP * 8];
  __shared__ int newf[kMaxKP], nnew;
  for (int c = lane; c < nc; c += 64) {
    const int j = c / KP, k = c % KP;
    const int r = r0 + j;
    cv[c] = rs.sum_lp[r] + clp[r * KP + k];
    cb[c] = j;
    ct[c] = ctok[r * KP + k];
  }
  __syncthreads();
  const int s = *slot;
  // rank sort, one candidate per lane (score desc, beam asc, token asc: a strict total order, since a beam's
  // candidate tokens are distinct): order[rank of c] = c
  for (int c = lane; c < nc; c += 64) {
    int rank = 0;
    for (int y = 0; y < nc; ++y)
      rank += cv[y] > cv[c] || (cv[y] == cv[c] && (cb[y] < cb[c] || (cb[y] == cb[c] && ct[y] < ct[c])));
    order[rank] = c;
  }
  __syncthreads();
  if (lane == 0) {
    bs.win_active[w] = 1;
    int saved = 0, nn = 0;
    int nf = bs.fin_count[w];
    for (int q = 0; q < nc && saved < K; ++q) {
      const int c = order[q];
      const int parent = r0 + cb[c];
      if (ct[c] == eot) {
        if (nf < max_cand) {
          const int f = w * max_cand + nf;
          bs.fin_score[f] = cv[c];
          bs.fin_parent[f] = parent;
          bs.fin_len[f] = s + 1;  // history slots [0, s] of the parent; EOT implied
          newf[nn++] = f;
          ++nf;
        }
      } else {
        bs.new_parent[r0 + saved] = parent;
        bs.new_tok[r0 + saved] = ct[c];
        bs.new_score[r0 + saved] = cv[c];
        ++saved;
      }
    }
    nnew = nn;
    bs.fin_count[w] = nf;
    if (nf >= max_cand) {
      bs.win_done[w] = 1;
      atomicAdd(n_done, 1);
    }
  }
  __syncthreads();
  // copy the histories of newly finished hypotheses (parents are still unmodified here)
  for (int q = 0; q < nnew; ++q) {
    const int f = newf[q];
    const int p = bs.fin_parent[f];
    for (int t = lane; t <= s; t += 64) bs.fin_hist[(long)f * hist_ld + t] = hist[(long)p * hist_ld + t];
  }
}

// block per row: new row r' <- parent history + token; ancestry row; state.  Windows inactive this step are frozen.
// beam update, one 1024-thread workgroup for all rows (so its barriers order the three phases): (1) copy each
// row's parent history / ancestry / rule state into the tmp rows, appending the new token at slot + 1; (2) copy
// the tmp rows back; (3) advance the slot once every thread has read it.  One launch instead of three.
constexpr int kBeamUpdThreads = 1024;
__global__ __launch_bounds__(kBeamUpdThreads) void beam_update_kernel(RowState rs, int R, int K, int tb,
                                                                      int* __restrict__ slot, int* __restrict__ hist,
                                                                      int* __restrict__ hist_tmp, int* __restrict__ anc,
                                                                      int* __restrict__ anc_tmp, int ld, BeamState bs,
                                                                      RowState tmp) {
  const int s = *slot;
  const int n = s + 1;  // history slots 0..s of every row
  for (int e = threadIdx.x; e < R * n; e += kBeamUpdThreads) {
    const int r = e / n, t = e - r * n;
    const int p = bs.win_active[r / K] ? bs.new_parent[r] : r;
    hist_tmp[(long)r * ld + t] = hist[(long)p * ld + t];
    anc_tmp[(long)r * ld + t] = anc[(long)p * ld + t];
  }
  if (threadIdx.x < R) {
    const int r = threadIdx.x;
    if (!bs.win_active[r / K]) {
      tmp.ns[r] = rs.ns[r];
      tmp.last[r] = rs.last[r];
      tmp.pen[r] = rs.pen[r];
      tmp.last_ts[r] = rs.last_ts[r];
      tmp.sum_lp[r] = rs.sum_lp[r];
      hist_tmp[(long)r * ld + s + 1] = 0;
    } else {
      const int p = bs.new_parent[r];
      const int t = bs.new_tok[r];
      hist_tmp[(long)r * ld + s + 1] = t;
      tmp.ns[r] = rs.ns[p] + 1;
      tmp.pen[r] = rs.last[p];
      tmp.last[r] = t;
      tmp.last_ts[r] = t >= tb ? t : rs.last_ts[p];
      tmp.sum_lp[r] = bs.new_score[r];
    }
    anc_tmp[(long)r * ld + s + 1] = r;
  }
  __syncthreads();  // workgroup-scope fence: the tmp rows are visible to every thread of the block
  const int n2 = s + 2;
  for (int e = threadIdx.x; e < R * n2; e += kBeamUpdThreads) {
    const int r = e / n2, t = e - r * n2;
    hist[(long)r * ld + t] = hist_tmp[(long)r * ld + t];
    anc[(long)r * ld + t] = anc_tmp[(long)r * ld + t];
  }
  if (threadIdx.x < R) {
    const int r = threadIdx.x;
    rs.ns[r] = tmp.ns[r];
    rs.last[r] = tmp.last[r];
    rs.pen[r] = tmp.pen[r];
    rs.last_ts[r] = tmp.last_ts[r];
    rs.sum_lp[r] = tmp.sum_lp[r];
  }
  __syncthreads();  // every thread has read *slot
  if (threadIdx.x == 0) *slot = s + 1;
}

// language detection: argmax over language tokens of the logits at <|startoftranscript|>; writes the token into
// the prompt of every row of the window
// (no finite language logit -- a NaN upstream: language 0 is written, so no id outside the vocabulary reaches the
// prefill's embedding gather, and the non-finite guard word gets -(1 + window), WMX_ERR_NUMERIC on the host)
__global__ void lang_detect_kernel(const float* __restrict__ logits, int ldl, int lang0, int nlang, int K,
                                   int* __restrict__ hist, int hist_ld, const int* __restrict__ lang_slot,
                                   int* __restrict__ lang_out, float* __restrict__ prob_out, int* __restrict__ err) {
  const int w = blockIdx.x;
  const float* x = logits + (long)w * ldl + lang0;
  const int lane = threadIdx.x;
  float bv = -INFINITY;
  int bi = 0x7FFFFFFF;
  for (int i = lane; i < nlang; i += 64)
    if (better(x[i], i, bv, bi)) {
      bv = x[i];
      bi = i;
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float v2 = __shfl_xor(bv, off);
    const int i2 = __shfl_xor(bi, off);
    if (better(v2, i2, bv, bi)) {
      bv = v2;
      bi = i2;
    }
  }
  if (bi < 0 || bi >= nlang) {  // (wave-uniform: every lane holds the reduced pair)
    bi = 0;
    if (lane == 0 && err) atomicCAS(err, 0, -(1 + w));
  }
  float s = 0.f;
  for (int i = lane; i < nlang; i += 64) s += __expf(x[i] - bv);
  s = wave_sum(s);
  if (lane == 0) {
    lang_out[w] = lang0 + bi;
    prob_out[w] = 1.0f / s;
  }
  if (hist && lane < K) hist[(long)(w * K + lane) * hist_ld + lang_slot[w]] = lang0 + bi;
}

// softmax(logits)[token] per row (no-speech probability at the SOT position)
__global__ void token_prob_kernel(const float* __restrict__ logits, int ldl, int V, int token, float* __restrict__ out) {
  const int r = blockIdx.x;
  const float* x = logits + (long)r * ldl;
  MS a{-INFINITY, 0.f};
  for (int t = threadIdx.x; t < V; t += 256) a = ms_add(a, x[t]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) a = ms_merge(a, MS{__shfl_xor(a.m, off), __shfl_xor(a.s, off)});
  __shared__ float sm[4], ss[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    sm[wave] = a.m;
    ss[wave] = a.s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MS t{-INFINITY, 0.f};
    for (int w = 0; w < 4; ++w) t = ms_merge(t, MS{sm[w], ss[w]});
    out[r] = __expf(x[token] - ms_lse(t));
  }
}

// text-token probabilities of the alignment forward: softmax over [0, eot) at row m, prob of target[m]
__global__ void text_prob_kernel(const float* __restrict__ logits, int ldl, int eot, const int* __restrict__ target,
                                 float* __restrict__ out) {
  const int r = blockIdx.x;
  const int tg = target[r];
  if (tg < 0) return;
  const float* x = logits + (long)r * ldl;
  MS a{-INFINITY, 0.f};
  for (int t = threadIdx.x; t < eot; t += 256) a = ms_add(a, x[t]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) a = ms_merge(a, MS{__shfl_xor(a.m, off), __shfl_xor(a.s, off)});
  __shared__ float sm[4], ss[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    sm[wave] = a.m;
    ss[wave] = a.s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MS t{-INFINITY, 0.f};
    for (int w = 0; w < 4; ++w) t = ms_merge(t, MS{sm[w], ss[w]});
    out[r] = __expf(x[tg] - ms_lse(t));
  }
}

// alignment matrix of one window: for every alignment head softmax over the first nf frames, normalise each frame
// column over the T tokens (population std), median filter (width W, reflect), mean over heads.
__device__ inline float median7(float* v, int n) {
  for (int i = 1; i < n; ++i) {
    const float x = v[i];
    int j = i - 1;
    while (j >= 0 && v[j] > x) {
      v[j + 1] = v[j];
      --j;
    }
    v[j + 1] = x;
  }
  return v[n / 2];
}

// alignment matrix of one decoder layer's alignment heads (faster-whisper/openai find_alignment), in three
// grid-wide passes over scores[hh][row][Tk] (rows = window * Tn + token), in place:
//   softmax over the window's nf = nframes/2 frames (one workgroup per (token, head, window)),
//   per-frame standardisation over the T tokens (one thread per frame),
//   median filter along frames, accumulated into out over the heads in head order.
__global__ __launch_bounds__(256) void align_softmax_kernel(float* __restrict__ scores, int rows_total, int Tk, int Tn,
                                                            const int* __restrict__ ntok,
                                                            const int* __restrict__ nframes) {
  const int t = blockIdx.x, hh = blockIdx.y, w = blockIdx.z;
  if (t >= ntok[w]) return;
  const int nf = nframes[w] / 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ float red[4];
  float* s = scores + ((long)hh * rows_total + (long)w * Tn + t) * Tk;
  float v[6];  // Tk <= 1536
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int f = tid + 256 * i;
    v[i] = f < nf ? s[f] : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int f = tid + 256 * i;
    v[i] = f < nf ? __expf(v[i] - mx) : 0.f;
    sum += v[i];
  }
  sum = wave_sum(sum);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  const float inv = 1.0f / (red[0] + red[1] + red[2] + red[3]);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int f = tid + 256 * i;
    if (f < nf) s[f] = v[i] * inv;
  }
}

// per (frame, alignment head, window): normalise the frame's column over the window's T tokens (mean, then centred
// variance, as openai timing.find_alignment).  Workgroup = 64 frames x 4 token groups: each thread walks every 4th
// token, 4 loads in flight, and the 4 partial sums meet in LDS (fixed order, so the result is deterministic).
__global__ __launch_bounds__(256) void align_colnorm_kernel(float* __restrict__ scores, int rows_total, int Tk, int Tn,
                                                            const int* __restrict__ ntok,
                                                            const int* __restrict__ nframes) {
  const int fl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + fl, hh = blockIdx.y, w = blockIdx.z;
  const int T = ntok[w], nf = nframes[w] / 2;
  if (T <= 0 || blockIdx.x * 64 >= nf) return;  // whole-block exit: every thread of it agrees
  const bool ok = f < nf;
  float* s = scores + ((long)hh * rows_total + (long)w * Tn) * Tk + (ok ? f : 0);
  __shared__ float red[4][64];
  auto colsum = [&](auto&& term) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int t = g;
    for (; t + 12 < T; t += 16) {
      a0 += term(s[(long)t * Tk]);
      a1 += term(s[(long)(t + 4) * Tk]);
      a2 += term(s[(long)(t + 8) * Tk]);
      a3 += term(s[(long)(t + 12) * Tk]);
    }
    for (; t < T; t += 4) a0 += term(s[(long)t * Tk]);
    red[g][fl] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    const float tot = (red[0][fl] + red[1][fl]) + (red[2][fl] + red[3][fl]);
    __syncthreads();
    return tot;
  };
  const float mean = colsum([](float v) { return v; }) / T;
  const float var = colsum([mean](float v) { return (v - mean) * (v - mean); }) / T;
  const float inv = 1.0f / sqrtf(var);
  if (ok)
    for (int t = g; t < T; t += 4) s[(long)t * Tk] = (s[(long)t * Tk] - mean) * inv;
}

__global__ __launch_bounds__(256) void align_median_acc_kernel(const float* __restrict__ scores, int nh, int rows_total,
                                                               int Tk, int Tn, const int* __restrict__ ntok,
                                                               const int* __restrict__ nframes, int width,
                                                               float* __restrict__ out) {
  const int t = blockIdx.x, w = blockIdx.y;
  if (t >= ntok[w]) return;
  const int nf = nframes[w] / 2, pad = width / 2;
  float* o = out + ((long)w * Tn + t) * Tk;
  for (int f = threadIdx.x; f < nf; f += 256) {
    float acc = o[f];
    for (int hh = 0; hh < nh; ++hh) {
      const float* sc = scores + ((long)hh * rows_total + (long)w * Tn + t) * Tk;
      float v;
      if (nf <= pad) {
        v = sc[f];
      } else {
        float win[15];
        for (int k = 0; k < width; ++k) {
          int j = f - pad + k;
          if (j < 0) j = -j;
          if (j >= nf) j = 2 * (nf - 1) - j;
          win[k] = sc[j];
        }
        v = median7(win, width);
      }
      acc += v;
    }
    o[f] = acc;
  }
}

// one workgroup per (token row, window): the row's frames scaled in place
__global__ void align_scale_kernel(float* __restrict__ out, int Tn, int Tk, const int* __restrict__ ntok,
                                   const int* __restrict__ nframes, float scale) {
  const int t = blockIdx.x, w = blockIdx.y;
  const int T = ntok[w], nf = nframes[w] / 2;
  if (t >= T) return;
  float* o = out + ((long)w * Tn + t) * Tk;
  for (int f = threadIdx.x; f < nf; f += 256) o[f] *= scale;
}

// ------------------------------------------------------------------------------------------------
size_t logits_select_ws_floats(int R, int KP) { return (size_t)R * kSlices * (5 + 4 * KP); }

void launch_logits_select(const float* logits, int ldl, const RuleOpts& o, const RowPtrs& rp, int R, int KP, int* tok,
                          float* lp, const int* row_map, float* ws, hipStream_t st) {
  WMX_CHECK(KP <= kMaxKP, "beam too large");
  WMX_CHECK(o.V <= kSlices * kSelPer && ldl % 2 == 0, "logits select: vocabulary / row stride");
  RowState rs{rp.ns, rp.last, rp.pen, rp.last_ts, rp.done, rp.sum_lp};
  if (o.inv_temp > 0.f) {  // sampling: one Gumbel-max draw per row
    WMX_CHECK(KP == 1 && o.slot && o.seed, "logits select: sampling draws one token per row");
    hipLaunchKernelGGL((logits_select_a<1, true>), dim3(R, kSlices), dim3(kSelA), 0, st, logits, ldl, o, rs, row_map, ws);
    hipLaunchKernelGGL((logits_select_b<1, true>), dim3(R), dim3(64), 0, st, ws, o, tok, lp, logits, ldl, row_map);
    WMX_HIP(hipGetLastError());
    return;
  }
  switch (KP) {
#define WMX_SEL_A(N)                                                                                             \
  case N:                                                                                                        \
    hipLaunchKernelGGL(logits_select_a<N>, dim3(R, kSlices), dim3(kSelA), 0, st, logits, ldl, o, rs, row_map, ws); \
    hipLaunchKernelGGL(logits_select_b<N>, dim3(R), dim3(64), 0, st, ws, o, tok, lp, logits, ldl, row_map);     \
    break;
    WMX_SEL_A(1)
    WMX_SEL_A(2)
    WMX_SEL_A(3)
    WMX_SEL_A(4)
    WMX_SEL_A(5)
    WMX_SEL_A(6)
    WMX_SEL_A(7)
    WMX_SEL_A(8)
    WMX_SEL_A(9)
#undef WMX_SEL_A
    default: WMX_CHECK(false, "logits select: list length");
  }
  WMX_HIP(hipGetLastError());
}

// ---- parity instrumentation (wmx_ctx_record): per decode step, the raw logits of every row before selection and
// the selection itself, at step index *slot - *base (- 1 after the update has advanced the slot) ----
__global__ void record_logits_kernel(const float* __restrict__ logits, int ldl, int V, int R, const int* __restrict__ row_map,
                                     const int* __restrict__ slot, const int* __restrict__ base, int cap,
                                     float* __restrict__ out) {
  const int r = blockIdx.y;
  const int idx = *slot - *base;
  if (idx < 0 || idx >= cap) return;
  const float* src = logits + (long)(row_map ? row_map[r] : r) * ldl;
  float* dst = out + ((long)idx * R + r) * V;
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) dst[v] = src[v];
}

// greedy (before the update): (row, first candidate) of live rows; beam (after the update): (parent, token) of the
// rows of windows active this step; (-1, -1) otherwise
__global__ void record_select_kernel(int R, int K, int KP, const int* __restrict__ ctok, const int* __restrict__ done,
                                     const int* __restrict__ win_active, const int* __restrict__ new_parent,
                                     const int* __restrict__ new_tok, const int* __restrict__ slot,
                                     const int* __restrict__ base, int after, int cap, int* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int idx = *slot - *base - after;
  if (r >= R || idx < 0 || idx >= cap) return;
  int p = -1, t = -1;
  if (K == 1) {
    if (!done[r]) {
      p = r;
      t = ctok[r * KP];
    }
  } else if (win_active[r / K]) {
    p = new_parent[r];
    t = new_tok[r];
  }
  out[((long)idx * R + r) * 2] = p;
  out[((long)idx * R + r) * 2 + 1] = t;
}

void launch_record_logits(const float* logits, int ldl, int V, int R, const int* row_map, const int* slot,
                          const int* base, int cap, float* out, hipStream_t st) {
  hipLaunchKernelGGL(record_logits_kernel, dim3(32, R), dim3(256), 0, st, logits, ldl, V, R, row_map, slot, base, cap,
                     out);
  WMX_HIP(hipGetLastError());
}

void launch_record_select(int R, int K, const int* ctok, const RowPtrs& rp, const BeamState& bs, const int* slot,
                          const int* base, int after, int cap, int* out, hipStream_t st) {
  hipLaunchKernelGGL(record_select_kernel, dim3((R + 255) / 256), dim3(256), 0, st, R, K, K + (K > 1 ? 1 : 0), ctok,
                     rp.done, bs.win_active, bs.new_parent, bs.new_tok, slot, base, after, cap, out);
  WMX_HIP(hipGetLastError());
}

void launch_greedy_update(const RowPtrs& rp, const int* tok, const float* lp, int R, int tb, int eot, int* hist,
                          int hist_ld, int* slot, int* n_done, hipStream_t st) {
  WMX_CHECK(R <= 1024, "greedy: too many rows");
  RowState rs{rp.ns, rp.last, rp.pen, rp.last_ts, rp.done, rp.sum_lp};
  hipLaunchKernelGGL(greedy_update_kernel, dim3(1), dim3(std::max(64, ((R + 63) / 64) * 64)), 0, st, rs, tok, lp, R, tb,
                     eot, hist, hist_ld, slot, n_done);
  WMX_HIP(hipGetLastError());
}

void launch_beam_step(const RowPtrs& rp, const RowPtrs& tmp, const int* ctok, const float* clp, int nwin, int K,
                      int max_cand, int tb, int eot, int* slot, int* hist, int* hist_tmp, int* anc, int* anc_tmp, int ld,
                      const BeamState& bs, int* n_done, hipStream_t st) {
  RowState rs{rp.ns, rp.last, rp.pen, rp.last_ts, rp.done, rp.sum_lp};
  RowState ts{tmp.ns, tmp.last, tmp.pen, tmp.last_ts, tmp.done, tmp.sum_lp};
  const int R = nwin * K;
  hipLaunchKernelGGL(beam_select_kernel, dim3(nwin), dim3(64), 0, st, rs, ctok, clp, K, max_cand, eot, slot, hist, ld, bs,
                     n_done);
  WMX_CHECK(R <= kBeamUpdThreads, "beam update: rows");
  hipLaunchKernelGGL(beam_update_kernel, dim3(1), dim3(kBeamUpdThreads), 0, st, rs, R, K, tb, slot, hist, hist_tmp,
                     anc, anc_tmp, ld, bs, ts);
  WMX_HIP(hipGetLastError());
}

void launch_lang_detect(const float* logits, int ldl, int lang0, int nlang, int nwin, int K, int* hist, int hist_ld,
                        const int* lang_slot, int* lang_out, float* prob_out, hipStream_t st, int* err) {
  hipLaunchKernelGGL(lang_detect_kernel, dim3(nwin), dim3(64), 0, st, logits, ldl, lang0, nlang, K, hist, hist_ld,
                     lang_slot, lang_out, prob_out, err);
  WMX_HIP(hipGetLastError());
}

void launch_token_prob(const float* logits, int ldl, int V, int token, int rows, float* out, hipStream_t st) {
  hipLaunchKernelGGL(token_prob_kernel, dim3(rows), dim3(256), 0, st, logits, ldl, V, token, out);
  WMX_HIP(hipGetLastError());
}

void launch_text_prob(const float* logits, int ldl, int eot, const int* target, int rows, float* out, hipStream_t st) {
  hipLaunchKernelGGL(text_prob_kernel, dim3(rows), dim3(256), 0, st, logits, ldl, eot, target, out);
  WMX_HIP(hipGetLastError());
}

void launch_align_matrix_zero(float* out, int nwin, int Tn, int Tk, hipStream_t st) {
  WMX_HIP(hipMemsetAsync(out, 0, (size_t)nwin * Tn * Tk * sizeof(float), st));
}

void launch_align_matrix_acc(float* scores, int nh, int rows_total, int Tk, int Tn, const int* ntok,
                             const int* nframes, int width, int nwin, hipStream_t st, float* out) {
  WMX_CHECK(width <= 15 && width % 2 == 1 && Tk <= 1536, "alignment: median filter width / frames");
  hipLaunchKernelGGL(align_softmax_kernel, dim3(Tn, nh, nwin), dim3(256), 0, st, scores, rows_total, Tk, Tn, ntok,
                     nframes);
  hipLaunchKernelGGL(align_colnorm_kernel, dim3((Tk + 63) / 64, nh, nwin), dim3(256), 0, st, scores, rows_total, Tk,
                     Tn, ntok, nframes);
  hipLaunchKernelGGL(align_median_acc_kernel, dim3(Tn, nwin), dim3(256), 0, st, scores, nh, rows_total, Tk, Tn, ntok,
                     nframes, width, out);
  WMX_HIP(hipGetLastError());
}

void launch_align_matrix_scale(float* out, int nwin, int Tn, int Tk, const int* ntok, const int* nframes, float scale,
                               hipStream_t st) {
  hipLaunchKernelGGL(align_scale_kernel, dim3(Tn, nwin), dim3(256), 0, st, out, Tn, Tk, ntok, nframes, scale);
  WMX_HIP(hipGetLastError());
}

}  // namespace wmx
