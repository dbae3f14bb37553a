// Beam search step on device (a10): GenerationMixin._beam_search (TF/generation/utils.py:3208-3527)
// for one decode step, captured in the same hipGraph as the decoder forward.
//
//  kw_beam_logprobs (one 1024-thread workgroup per running row = batch item x beam):
//    log_softmax of the raw f32 logits (:3380), the Whisper processors on the log-probs (Suppress ->
//    SuppressAtBegin -> WhisperTimeStamp, processors.h; :3381), and the row's K best processed
//    log-probs (K = 2 * num_beams: the global top-K over beams x vocab of log-prob + beam score is
//    always inside the union of the rows' top-K, adding a per-row constant keeps a row's order).
//  kw_beam_select (one workgroup per batch item):
//    _get_top_k_continuations (:3077), the MaxLength / EOS stopping criteria on the K continuations,
//    _get_running_beams_for_next_iteration (:3131), _update_finished_beams (:3153, length penalty,
//    early_stopping), the cache reorder (:3445-3456) and _check_early_stop_heuristic (:3008) /
//    _beam_search_has_unfinished_sequences (:3055).  The reorder moves no K/V: every running row
//    keeps a slot table bp[row][pos] = the cache row that holds its position pos (a beam's history
//    is its parent's table + its own new slot), so a reorder rewrites nb x L int32 per item
//    instead of gathering nb x layers x heads x L x 64 K/V values.
// All arithmetic is fp32 in the reference's order (log-prob + score, -1e9 masks, score /
// len**length_penalty); every top-k breaks ties by the lower flat index.
#include <math.h>

#include "processors.h"

namespace {

using namespace kwp;

constexpr int KMAX = 16;  // candidates per row (2 * num_beams <= 16)
constexpr float NEG = -1.0e9f;

__device__ __forceinline__ bool better(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }

// (score, token) as one 64-bit key ordered like better(): monotonic float bits above, ~token below.
// -0 is folded into +0 first (better() compares values).  Key 0 = no candidate.
__device__ __forceinline__ uint64_t bkey(float s, int v) {
  uint32_t b = __float_as_uint(s + 0.0f);
  b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return ((uint64_t)b << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)v);
}
__device__ __forceinline__ float bkey_val(uint64_t k) {
  const uint32_t b = (uint32_t)(k >> 32);
  return __uint_as_float((b & 0x80000000u) ? (b & 0x7fffffffu) : ~b);
}
__device__ __forceinline__ int bkey_idx(uint64_t k) { return (int)(0xFFFFFFFFu - (uint32_t)k); }
// insert k into the descending triple (c0, c1, c2)
__device__ __forceinline__ void bins3(uint64_t k, uint64_t& c0, uint64_t& c1, uint64_t& c2) {
  const uint64_t h0 = k > c0 ? k : c0, l0 = k > c0 ? c0 : k;
  const uint64_t h1 = l0 > c1 ? l0 : c1, l1 = l0 > c1 ? c1 : l0;
  c0 = h0;
  c1 = h1;
  c2 = l1 > c2 ? l1 : c2;
}
// wave maximum of 64-bit keys on the VALU: DPP within 16-lane rows (quad_perm ^1 / ^2, then half-row and
// row mirrors once the quads / halves are uniform), v_permlane16/32_swap across rows -- no ds_bpermute round
// trips (a maximum is exact, so any reduction tree gives the butterfly's result)
template <int CTRL>
__device__ __forceinline__ uint64_t u64_max_dpp(uint64_t k) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(k >> 32), CTRL, 0xF, 0xF, false);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)k, CTRL, 0xF, 0xF, false);
  const uint64_t o = ((uint64_t)hi << 32) | lo;
  return o > k ? o : k;
}
__device__ __forceinline__ uint64_t u64_max_swap16(uint64_t k) {
  const auto h = __builtin_amdgcn_permlane16_swap((uint32_t)(k >> 32), (uint32_t)(k >> 32), false, false);
  const auto l = __builtin_amdgcn_permlane16_swap((uint32_t)k, (uint32_t)k, false, false);
  const uint64_t a = ((uint64_t)h[0] << 32) | l[0], b = ((uint64_t)h[1] << 32) | l[1];
  return a > b ? a : b;
}
__device__ __forceinline__ uint64_t u64_max_swap32(uint64_t k) {
  const auto h = __builtin_amdgcn_permlane32_swap((uint32_t)(k >> 32), (uint32_t)(k >> 32), false, false);
  const auto l = __builtin_amdgcn_permlane32_swap((uint32_t)k, (uint32_t)k, false, false);
  const uint64_t a = ((uint64_t)h[0] << 32) | l[0], b = ((uint64_t)h[1] << 32) | l[1];
  return a > b ? a : b;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t k) {
  k = u64_max_dpp<0xB1>(k);   // quad_perm [1,0,3,2]
  k = u64_max_dpp<0x4E>(k);   // quad_perm [2,3,0,1]
  k = u64_max_dpp<0x141>(k);  // row_half_mirror
  k = u64_max_dpp<0x140>(k);  // row_mirror
  return u64_max_swap32(u64_max_swap16(k));
}

// The wave's best key, exactly wave_max_u64(k), at about a third of its VALU: a 32-bit maximum of the keys'
// value words (one v_max_u32 per DPP / swap step instead of a 64-bit compare and two selects), a ballot of the
// lanes that hold it, and the holder's key by readlane; only a tie on the value (several lanes, one value)
// falls back to the 64-bit maximum over those lanes (the lowest token among them).  Value words are never 0
// for a key (bkey's monotonic bits of any non-NaN score are >= 0x007FFFFF); key 0 = no candidate.
template <int CTRL>
__device__ __forceinline__ uint32_t u32_max_dpp(uint32_t v) {
  const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
  return o > v ? o : v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = u32_max_dpp<0xB1>(v);
  v = u32_max_dpp<0x4E>(v);
  v = u32_max_dpp<0x141>(v);
  v = u32_max_dpp<0x140>(v);
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = a[0] > a[1] ? a[0] : a[1];
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return b[0] > b[1] ? b[0] : b[1];
}
__device__ __forceinline__ uint64_t wave_best_key(uint64_t k) {
  const uint32_t hi = (uint32_t)(k >> 32);
  const uint32_t gh = wave_max_u32(hi);
  const uint64_t hit = __ballot(hi == gh && gh != 0);
  if (hit == 0) return 0;
  if (hit & (hit - 1)) return wave_max_u64(hi == gh ? k : 0);
  const int w = __builtin_ctzll(hit);
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, w) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, w);
}

__global__ __launch_bounds__(ST) void beam_logprobs_kernel(kw_beam_logprobs_args a) {
  __shared__ float shf[ST / 64];
  __shared__ int shi[ST / 64][2];
  __shared__ RowState st_sh;
  __shared__ int win_t;
  if (*a.done) return;
  const int r = blockIdx.x;
  const int tid = threadIdx.x;
  const int L = *a.cur_len;
  const int V = (int)a.V;
  const int K = a.k;
  const float* x = a.logits + (int64_t)r * a.V;
  const int64_t* ids = a.ids + (int64_t)r * a.ids_stride;

  // log_softmax normaliser of the raw row: lp = (x - max) - log(sum exp(x - max))
  float m = -INFINITY;
#pragma unroll 8
  for (int v = tid; v < V; v += ST) m = fmaxf(m, x[v]);
  m = block_reduce_max(m, shf);
  float s = 0.f;
#pragma unroll 8
  for (int v = tid; v < V; v += ST) s += expf(x[v] - m);
  s = block_reduce_sum(s, shf);
  const float ls = logf(s);
  auto lp = [&](int v) { return (x[v] - m) - ls; };

  int fin = 0;
  RowState st = row_state(ids, L, a.begin_index, a.ts_begin, a.no_ts_id, a.eos_id, a.return_timestamps,
                          a.max_initial_ts, &fin, shi, &st_sh);
  if (st.rt) timestamp_rule(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, V, lp, shf);

  // per-thread sorted top-K of its strided slice, then K rounds of a block arg-max over the heads
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    tv[i] = -INFINITY;
    ti[i] = 0x7fffffff;
  }
  for (int v = tid; v < V; v += ST) {
    const float sv = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, lp(v));
    if (!better(sv, v, tv[KMAX - 1], ti[KMAX - 1])) continue;  // (keeps KMAX >= K per thread)
    // insert (v increases along the slice, so an equal value goes after the existing ones)
    float cv = sv;
    int ci = v;
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      if (better(cv, ci, tv[i], ti[i])) {
        const float t1 = tv[i];
        const int t2 = ti[i];
        tv[i] = cv;
        ti[i] = ci;
        cv = t1;
        ci = t2;
      }
    }
  }
  int head = 0;
  for (int k = 0; k < K; ++k) {
    float hv = -INFINITY;
    int hi = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < KMAX; ++i)
      if (i == head) {
        hv = tv[i];
        hi = ti[i];
      }
    float bv = hv;
    int bi = hi, bt = tid;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64), ot = __shfl_xor(bt, o, 64);
      if (better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
        bt = ot;
      }
    }
    if ((tid & 63) == 0) {
      shf[tid >> 6] = bv;
      shi[tid >> 6][0] = bi;
      shi[tid >> 6][1] = bt;
    }
    __syncthreads();
    if (tid == 0) {
      float gv = shf[0];
      int gi = shi[0][0], gt = shi[0][1];
      for (int w = 1; w < ST / 64; ++w)
        if (better(shf[w], shi[w][0], gv, gi)) {
          gv = shf[w];
          gi = shi[w][0];
          gt = shi[w][1];
        }
      a.cand_val[(int64_t)r * K + k] = gv;
      a.cand_idx[(int64_t)r * K + k] = gi == 0x7fffffff ? 0 : gi;
      win_t = gt;
    }
    __syncthreads();
    if (tid == win_t) ++head;
    __syncthreads();
  }
}

// ---- split-row variant: a row over BSPLIT workgroups (the one-workgroup kernel above walks a whole
// vocabulary row serially in several passes; at R = 160-320 running rows that is most of a step).
// Each slice keeps its logits in registers and publishes: the raw maximum and sum of exp (the
// log_softmax normaliser), WhisperTimeStamp's statistics of its processed scores (as the greedy
// split kernel), and its best KP processed scores overall and among timestamps (KP = k + 4 > k, so a
// log-prob tie that the raw order would split differently stays inside the candidates).  The row's
// last arriver merges the normaliser, applies the timestamp rule, turns candidates into log-probs
// lp = (x - m) - log(s) and keeps the k best by (lp desc, token asc).
constexpr int BSPLIT = 8, BT_S = 512, BUNR = 16, KP = KMAX + 4, BPART = 96;

__device__ __forceinline__ void bl_argmax(float& best, int& bi, int& bt, float* shf, int* shi) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64), ot = __shfl_xor(bt, o, 64);
    if (better(ob, oi, best, bi)) { best = ob; bi = oi; bt = ot; }
  }
  if ((threadIdx.x & 63) == 0) {
    shf[threadIdx.x >> 6] = best;
    shi[2 * (threadIdx.x >> 6)] = bi;
    shi[2 * (threadIdx.x >> 6) + 1] = bt;
  }
  __syncthreads();
  best = shf[0]; bi = shi[0]; bt = shi[1];
  for (int w = 1; w < BT_S / 64; ++w)
    if (better(shf[w], shi[2 * w], best, bi)) { best = shf[w]; bi = shi[2 * w]; bt = shi[2 * w + 1]; }
  __syncthreads();
}
__device__ __forceinline__ float bl_max(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < BT_S / 64; ++i) r = fmaxf(r, sh[i]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ float bl_sum(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < BT_S / 64; ++i) r += sh[i];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(BT_S) void beam_logprobs_split_kernel(kw_beam_logprobs_args a) {
  __shared__ RowState st_sh;
  __shared__ float pub[BPART];
  if (*a.done) return;
  const int r = blockIdx.x, sl = blockIdx.y;
  const int tid = threadIdx.x;
  const int L = *a.cur_len;
  const int V = (int)a.V;
  const int K = a.k;
  const float* x = a.logits + (int64_t)r * a.V;
  const int64_t* ids = a.ids + (int64_t)r * a.ids_stride;
  const int per = (V + BSPLIT - 1) / BSPLIT;
  const int v0 = sl * per, v1 = min(V, v0 + per);
  float xv[BUNR];
  bool mk[BUNR];  // SuppressTokens bytes with the logits (a mask load in the compare chain waits per element)
#pragma unroll
  for (int u = 0; u < BUNR; ++u) {
    const int v = v0 + tid + u * BT_S, vc = min(v, v1 - 1);  // unconditional (clamped) loads: no branches
    const float xr = x[vc];                                           // and phis between them
    const uint8_t mr = a.suppress_mask[vc];
    xv[u] = v < v1 ? xr : -INFINITY;
    mk[u] = v < v1 ? mr != 0 : true;
  }
  // row state from the history (as kwp::row_state, BT_S threads): the last timestamp position travels with
  // its token in one 64-bit key (no dependent reload), the last two tokens are read up front
  const int n_hist = L - a.begin_index;
  const int64_t tok_l1 = n_hist >= 1 ? ids[L - 1] : 0, tok_l2 = n_hist >= 2 ? ids[L - 2] : 0;
  uint64_t lkey = 0;  // ((position + 1) << 32) | token of the row's last timestamp
  for (int p = a.begin_index + tid; p < L; p += BT_S) {
    const int64_t t = ids[p];
    if (t >= a.ts_begin) lkey = ((uint64_t)(uint32_t)(p + 1) << 32) | (uint32_t)t;
  }
  lkey = wave_max_u64(lkey);
  __shared__ uint64_t lkeys[BT_S / 64];
  if ((tid & 63) == 0) lkeys[tid >> 6] = lkey;
  __syncthreads();
  if (tid == 0) {
    uint64_t lk = lkeys[0];
    for (int i = 1; i < BT_S / 64; ++i) lk = lkeys[i] > lk ? lkeys[i] : lk;
    const int lp = (int)(lk >> 32) - 1;
    const int lp_tok = (int)(uint32_t)lk;
    RowState st;
    st.L = L; st.begin = a.begin_index; st.ts_begin = a.ts_begin; st.no_ts = a.no_ts_id; st.eos = a.eos_id;
    st.rt = a.return_timestamps; st.max_init = a.max_initial_ts; st.ban_text = 0;
    st.first_step = (L == a.begin_index);
    st.last_ts = n_hist >= 1 && tok_l1 >= a.ts_begin;
    st.pen_ts = n_hist < 2 || tok_l2 >= a.ts_begin;
    st.has_stamp = lp >= 0;
    st.stamp_lo = st.has_stamp ? ((st.last_ts && !st.pen_ts) ? lp_tok : lp_tok + 1) : 0;
    st_sh = st;
  }
  __syncthreads();
  const RowState st = st_sh;
  // processed scores (raw-logit space; every processor is shift invariant) and their statistics
  float sv[BUNR];
  float mr = -INFINITY, mt = -INFINITY, ms = -INFINITY;
  int it = 0x7fffffff, is = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < BUNR; ++u) {
    const int v = v0 + tid + u * BT_S;
    mr = fmaxf(mr, xv[u]);
    sv[u] = v < v1 ? process_m(st, mk[u], a.begin_suppress, a.n_begin_suppress, v, xv[u]) : -INFINITY;
    if (v < v1) {
      if (v < st.ts_begin) {
        if (better(sv[u], v, mt, it)) { mt = sv[u]; it = v; }
      } else if (better(sv[u], v, ms, is)) { ms = sv[u]; is = v; }
    }
  }
  // one workgroup round for the three maxima (the raw maximum of the log_softmax normaliser; the best
  // text and timestamp scores as 64-bit keys), one for the three sums
  __shared__ float rmx[BT_S / 64];
  __shared__ uint64_t rkt[BT_S / 64], rks[BT_S / 64];
  __shared__ float rsum[3][BT_S / 64];
  {
    mr = wave_max(mr);
    uint64_t kt = 0, ks = 0;
    if (st.rt) {
      kt = wave_max_u64(bkey(mt, it));
      ks = wave_max_u64(bkey(ms, is));
    }
    if ((tid & 63) == 0) { rmx[tid >> 6] = mr; rkt[tid >> 6] = kt; rks[tid >> 6] = ks; }
    __syncthreads();
    mr = rmx[0];
    kt = rkt[0];
    ks = rks[0];
    for (int w = 1; w < BT_S / 64; ++w) {
      mr = fmaxf(mr, rmx[w]);
      kt = rkt[w] > kt ? rkt[w] : kt;
      ks = rks[w] > ks ? rks[w] : ks;
    }
    if (st.rt) {
      mt = bkey_val(kt); it = bkey_idx(kt);
      ms = bkey_val(ks); is = bkey_idx(ks);
    }
  }
  float sr = 0.f, sa = 0.f, sts = 0.f, mall = -INFINITY;
  if (st.rt) mall = fmaxf(mt, ms);
#pragma unroll
  for (int u = 0; u < BUNR; ++u) {
    const int v = v0 + tid + u * BT_S;
    if (v < v1) {
      sr += expf(xv[u] - mr);
      if (mall > -INFINITY && sv[u] > -INFINITY) {
        sa += expf(sv[u] - mall);
        if (v >= st.ts_begin) sts += expf(sv[u] - ms);
      }
    }
  }
  {
    sr = wave_sum(sr);
    sa = wave_sum(sa);
    sts = wave_sum(sts);
    if ((tid & 63) == 0) { rsum[0][tid >> 6] = sr; rsum[1][tid >> 6] = sa; rsum[2][tid >> 6] = sts; }
    __syncthreads();
    sr = sa = sts = 0.f;
    for (int w = 0; w < BT_S / 64; ++w) {
      sr += rsum[0][w];
      sa += rsum[1][w];
      sts += rsum[2][w];
    }
  }
  // the slice's KP best processed scores (all tokens; and timestamps only, for the text-ban case):
  // each wave takes its own kp best by shuffle-only rounds (no workgroup barrier per round), then wave 0
  // takes the slice's kp best of the waves' 8 x kp
  const int kp = min(K + 4, KP);
  const int lane = tid & 63, wv = tid >> 6;
  __shared__ uint64_t wck[2][BT_S / 64][KP];
  // timestamp tokens sit at the top of the vocabulary: only the slices holding some need the second list
  const int nlist = (st.rt && v1 > st.ts_begin) ? 2 : 1;
  for (int list = 0; list < nlist; ++list) {
    // each lane keeps its 3 best keys below ``floor`` (the last key it gave up), refilled from its 16
    // registers in the rare round that empties it; a round is one wave max of the lanes' heads
    uint64_t c0 = 0, c1 = 0, c2 = 0, floor = ~0ull;
    auto fill = [&]() {
      c0 = c1 = c2 = 0;
#pragma unroll
      for (int u = 0; u < BUNR; ++u) {
        const int v = v0 + tid + u * BT_S;
        const uint64_t k = (v < v1 && (list == 0 || v >= st.ts_begin)) ? bkey(sv[u], v) : 0;
        if (k < floor) bins3(k, c0, c1, c2);
      }
    };
    fill();
    for (int j = 0; j < kp; ++j) {
      const uint64_t g = wave_best_key(c0);
      if (lane == 0) wck[list][wv][j] = g;
      bool need = false;
      if (g != 0 && c0 == g) {
        floor = g;
        c0 = c1; c1 = c2; c2 = 0;
        need = c0 == 0;
      }
      if (__ballot(need)) {
        if (need) fill();
      }
    }
  }
  __syncthreads();
  if (wv == 0) {
    for (int list = 0; list < 2; ++list) {
      if (list >= nlist) {  // (no timestamp tokens in this slice: an empty list)
        if (lane < kp) {
          pub[9 + list * 2 * KP + 2 * lane] = -INFINITY;
          pub[9 + list * 2 * KP + 2 * lane + 1] = __int_as_float(0x7fffffff);
        }
        continue;
      }
      // the waves' 8 x kp keys (kp <= KP: at most 3 per lane), then kp rounds of a wave max
      uint64_t c0 = 0, c1 = 0, c2 = 0;
      const int n = (BT_S / 64) * kp;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int e = lane + 64 * t;
        if (e < n) bins3(wck[list][e / kp][e % kp], c0, c1, c2);
      }
      for (int j = 0; j < kp; ++j) {
        const uint64_t g = wave_best_key(c0);
        if (g != 0 && c0 == g) { c0 = c1; c1 = c2; c2 = 0; }
        if (lane == 0) {
          pub[9 + list * 2 * KP + 2 * j] = g ? bkey_val(g) : -INFINITY;
          pub[9 + list * 2 * KP + 2 * j + 1] = __int_as_float(g ? bkey_idx(g) : 0x7fffffff);
        }
      }
    }
  }
  if (tid == 0) {
    pub[0] = mr; pub[1] = sr; pub[2] = mt; pub[3] = __int_as_float(it); pub[4] = ms;
    pub[5] = __int_as_float(is); pub[6] = mall; pub[7] = sa; pub[8] = sts;
  }
  __syncthreads();
  float* part = reinterpret_cast<float*>(a.workspace) + ((int64_t)r * BSPLIT + sl) * BPART;
  int* rcnt = reinterpret_cast<int*>(a.workspace) + (int64_t)a.R * BSPLIT * BPART + r;
  const int npub = 9 + (st.rt ? 4 : 2) * KP;
  if (tid < npub) __hip_atomic_store(part + tid, pub[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(rcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == BSPLIT - 1;
    if (last) __hip_atomic_store(rcnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  // the row's partials into LDS by the whole workgroup (one round trip), then one thread merges
  __shared__ float allp[BSPLIT * BPART];
  const float* row = reinterpret_cast<const float*>(a.workspace) + (int64_t)r * BSPLIT * BPART;
  for (int i = tid; i < BSPLIT * BPART; i += BT_S)
    allp[i] = (i % BPART) < npub ? __hip_atomic_load(row + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
  __syncthreads();
  if (wv != 0) return;
  // wave 0 merges: every lane derives the row's normaliser and the text-ban decision from the BSPLIT
  // slice records (identical on all lanes), then k rounds of a wave arg-max pick the candidates
  auto ld = [&](int q, int i) { return allp[q * BPART + i]; };
  float m = -INFINITY;
  for (int q = 0; q < BSPLIT; ++q) m = fmaxf(m, ld(q, 0));
  float ssum = 0.f;
  for (int q = 0; q < BSPLIT; ++q) {
    const float mq = ld(q, 0);
    if (mq > -INFINITY) ssum += ld(q, 1) * expf(mq - m);
  }
  const float ls = logf(ssum);
  int ban = 0;
  if (st.rt) {
    float bt_ = -INFINITY, bs_ = -INFINITY, M = -INFINITY;
    int jt = 0x7fffffff, js = 0x7fffffff;
    for (int q = 0; q < BSPLIT; ++q) {
      if (better(ld(q, 2), __float_as_int(ld(q, 3)), bt_, jt)) { bt_ = ld(q, 2); jt = __float_as_int(ld(q, 3)); }
      if (better(ld(q, 4), __float_as_int(ld(q, 5)), bs_, js)) { bs_ = ld(q, 4); js = __float_as_int(ld(q, 5)); }
      M = fmaxf(M, ld(q, 6));
    }
    float S = 0.f, Sts = 0.f;
    for (int q = 0; q < BSPLIT; ++q) {
      if (ld(q, 6) > -INFINITY) S += ld(q, 7) * expf(ld(q, 6) - M);
      if (ld(q, 4) > -INFINITY) Sts += ld(q, 8) * expf(ld(q, 4) - bs_);
    }
    if (M > -INFINITY) {
      const float lse = logf(S);
      const float lp_text_max = (bt_ - M) - lse;
      const float lp_ts_max = (bs_ - M) - lse;
      const float ts_lse = lp_ts_max > -INFINITY ? lp_ts_max + logf(Sts) : -INFINITY;
      ban = ts_lse > lp_text_max;
    }
  }
  // candidates of the chosen list as log-probs, three per lane (BSPLIT x kp <= 192)
  const int base = 9 + (ban ? 2 * KP : 0);
  const int n = BSPLIT * kp;
  float c[3];
  int ci3[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int e = lane + 64 * t;
    c[t] = -INFINITY;
    ci3[t] = 0x7fffffff;
    if (e < n) {
      const int q = e / kp, j = e - q * kp;
      const float sval = ld(q, base + 2 * j);
      const int idx = __float_as_int(ld(q, base + 2 * j + 1));
      if (idx != 0x7fffffff) {
        c[t] = sval > -INFINITY ? (sval - m) - ls : -INFINITY;
        ci3[t] = idx;
      }
    }
  }
  // k rounds of a wave maximum over 64-bit (log-prob, token) keys ordered like better() (token indices are
  // unique, so exactly one lane holds the winner; it writes its own f32 value and retires the key)
  uint64_t kk[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) kk[t] = ci3[t] != 0x7fffffff ? bkey(c[t], ci3[t]) : 0;
  for (int j = 0; j < K; ++j) {
    uint64_t b = kk[0] > kk[1] ? kk[0] : kk[1];
    b = b > kk[2] ? b : kk[2];
    const uint64_t g = wave_best_key(b);
    if (g == 0) {  // no candidate left (cannot happen with a sane config): as the reference's -inf / 0
      if (lane == 0) {
        a.cand_val[(int64_t)r * K + j] = -INFINITY;
        a.cand_idx[(int64_t)r * K + j] = 0;
      }
      continue;
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
      if (kk[t] == g) {
        a.cand_val[(int64_t)r * K + j] = c[t];
        a.cand_idx[(int64_t)r * K + j] = ci3[t];
        kk[t] = 0;
      }
  }
}

// K rounds of a block arg-max over n (value, key) pairs in LDS; writes the winners' positions in order.
__device__ void block_topk(const float* val, const int* key, int n, int k, int* out_pos, float* shf, int* shi) {
  const int tid = threadIdx.x;
  __shared__ int taken[256];
  for (int i = tid; i < n; i += blockDim.x) taken[i] = 0;
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    float bv = -INFINITY;
    int bk = 0x7fffffff, bp = -1;
    for (int i = tid; i < n; i += blockDim.x)
      if (!taken[i] && (bp < 0 || better(val[i], key[i], bv, bk))) {
        bv = val[i];
        bk = key[i];
        bp = i;
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int ok = __shfl_xor(bk, o, 64), op = __shfl_xor(bp, o, 64);
      if (op >= 0 && (bp < 0 || better(ov, ok, bv, bk))) {
        bv = ov;
        bk = ok;
        bp = op;
      }
    }
    if ((tid & 63) == 0) {
      shf[tid >> 6] = bv;
      shi[2 * (tid >> 6)] = bk;
      shi[2 * (tid >> 6) + 1] = bp;
    }
    __syncthreads();
    if (tid == 0) {
      float gv = shf[0];
      int gk = shi[0], gp = shi[1];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
        const int wp = shi[2 * w + 1];
        if (wp >= 0 && (gp < 0 || better(shf[w], shi[2 * w], gv, gk))) {
          gv = shf[w];
          gk = shi[2 * w];
          gp = wp;
        }
      }
      out_pos[j] = gp;
      taken[gp] = 1;
    }
    __syncthreads();
  }
}

constexpr int BT = 256;  // beam_select threads
constexpr int NBMAX = 8;
constexpr int TMAX = 512;  // history length bound (max_target_positions 448)

__global__ __launch_bounds__(BT) void beam_select_kernel(kw_beam_select_args a) {
  __shared__ float cval[256];
  __shared__ int ckey[256];
  __shared__ float shf[BT / 64];
  __shared__ int shi[2 * (BT / 64)];
  __shared__ int top[KMAX], run_pos[NBMAX], fin_pos[NBMAX];
  __shared__ float t_lp[KMAX], t_run[KMAX], t_fin[KMAX];
  __shared__ int t_par[KMAX], t_tok[KMAX], t_hit[KMAX];
  __shared__ float m_val[NBMAX + KMAX];
  __shared__ int m_key[NBMAX + KMAX];
  __shared__ float old_fs[NBMAX];
  __shared__ int old_fl[NBMAX], old_ff[NBMAX];
  __shared__ int hist[NBMAX][TMAX];  // parents' token histories (ids < 2^31)
  __shared__ int bph[NBMAX][TMAX];   // parents' slot tables
  __shared__ int fst[NBMAX][TMAX];   // the item's finished rows before this step
  __shared__ int last;
  if (*a.done) return;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nb = a.num_beams, K = 2 * nb;
  const int L = *a.cur_len, P = a.begin_index;
  const int V = (int)a.V;
  const int r0 = b * nb;

  // 1. candidates: row j's K processed log-probs + its running score; key = flat index j*V + v
  const int n = nb * K;
  for (int i = tid; i < n; i += BT) {
    const int j = i / K;
    cval[i] = a.cand_val[(int64_t)(r0 + j) * K + (i - j * K)] + a.run_scores[r0 + j];
    ckey[i] = j * V + a.cand_idx[(int64_t)(r0 + j) * K + (i - j * K)];
  }
  for (int i = tid; i < nb; i += BT) {
    old_fs[i] = a.fin_score[(int64_t)b * nb + i];
    old_fl[i] = a.fin_len[(int64_t)b * nb + i];
    old_ff[i] = a.fin_flag[(int64_t)b * nb + i];
  }
  // parents' histories (positions < L) and slot tables, before anything is rewritten
  for (int i = tid; i < nb * L; i += BT) {
    const int j = i / L, p = i - j * L;
    hist[j][p] = (int)a.ids[(int64_t)(r0 + j) * a.ids_stride + p];
    if (a.bp) bph[j][p] = a.bp[(int64_t)(r0 + j) * a.bp_stride + p];
  }
  __syncthreads();
  // 2. top-K continuations (:3077-3129)
  block_topk(cval, ckey, n, K, top, shf, shi);
  const bool at_max = L + 1 >= a.max_length;
  if (tid < K) {
    const int i = top[tid];
    t_lp[tid] = cval[i];
    t_par[tid] = ckey[i] / V;
    t_tok[tid] = ckey[i] - (ckey[i] / V) * V;
    const int hit = at_max || t_tok[tid] == a.eos_id;  // MaxLength / EOS criteria on the new sequence
    t_hit[tid] = hit;
    t_run[tid] = t_lp[tid] + (hit ? 1.f : 0.f) * NEG;  // :3144
  }
  __syncthreads();
  // 3. running beams for the next step (:3131-3151): top nb of t_run, key = candidate rank
  if (tid < K) {
    cval[tid] = t_run[tid];
    ckey[tid] = tid;
  }
  __syncthreads();
  block_topk(cval, ckey, K, nb, run_pos, shf, shi);
  // 4. finished beams (:3153-3205)
  if (tid == 0) {
    int all_fin = 1;
    for (int j = 0; j < nb; ++j) all_fin &= old_ff[j] != 0;
    const float full = (all_fin && a.early_stopping == 1) ? 1.f : 0.f;
    const float unsat0 = a.unsat[b] ? 0.f : 1.f;  // (~unsat) as f32
    const float den = (float)pow((double)(L + 1 - P), (double)a.length_penalty);
    for (int c = 0; c < K; ++c) {
      const int did = t_hit[c] && c < nb;
      float tl = t_lp[c] / den;
      tl = tl + full * NEG;
      tl = tl + unsat0 * NEG;
      tl = tl + (did ? 0.f : 1.f) * NEG;
      t_fin[c] = tl;
    }
    for (int j = 0; j < nb; ++j) {
      m_val[j] = old_fs[j];
      m_key[j] = j;
    }
    for (int c = 0; c < K; ++c) {
      m_val[nb + c] = t_fin[c];
      m_key[nb + c] = nb + c;
    }
  }
  __syncthreads();
  block_topk(m_val, m_key, nb + K, nb, fin_pos, shf, shi);
  // 5. the new finished set: old entries come from the LDS copy, new ones are a candidate's parent
  //    history + its token, fill (pad) beyond -- as the reference's static-shape sequences
  const int Tf = (int)a.fin_stride;
  for (int i = tid; i < nb * Tf; i += BT) {
    const int j = i / Tf, p = i - j * Tf;
    fst[j][p] = (int)a.fin_seq[((int64_t)b * nb + j) * Tf + p];
  }
  __shared__ int fin_src[NBMAX];
  if (tid < nb) fin_src[tid] = fin_pos[tid];
  __syncthreads();
  for (int i = tid; i < nb * Tf; i += BT) {
    const int s = i / Tf, p = i - s * Tf;
    const int src = fin_src[s];
    int v;
    if (src < nb) {
      v = fst[src][p];
    } else {
      const int c = src - nb;
      v = p < L ? hist[t_par[c]][p] : (p == L ? t_tok[c] : a.fill_id);
    }
    a.fin_seq[((int64_t)b * nb + s) * Tf + p] = v;
  }
  if (tid < nb) {
    const int src = fin_src[tid];
    float fs;
    int fl, ff;
    if (src < nb) {
      fs = old_fs[src];
      fl = old_fl[src];
      ff = old_ff[src];
    } else {
      fs = t_fin[src - nb];
      fl = L + 1 - P;
      ff = t_hit[src - nb] && (src - nb) < nb;
    }
    a.fin_score[(int64_t)b * nb + tid] = fs;
    a.fin_len[(int64_t)b * nb + tid] = fl;
    a.fin_flag[(int64_t)b * nb + tid] = ff;
  }
  // 6. running rows: parent history + new token, slot table of the parent + own slot at L
  for (int i = tid; i < nb * (L + 1); i += BT) {
    const int j = i / (L + 1), p = i - j * (L + 1);
    const int c = run_pos[j];
    a.ids[(int64_t)(r0 + j) * a.ids_stride + p] = p < L ? hist[t_par[c]][p] : (int64_t)t_tok[c];
    if (a.bp) a.bp[(int64_t)(r0 + j) * a.bp_stride + p] = p < L ? bph[t_par[c]][p] : r0 + j;
  }
  if (tid < nb) a.run_scores[r0 + tid] = t_run[run_pos[tid]];
  __syncthreads();
  // 7. early-stop heuristic (:3008-3053) at cur_len + 1, and this item's loop-condition inputs
  if (tid == 0) {
    const int Ln = L + 1;
    const int bhl = (a.early_stopping == 2 && a.length_penalty > 0.f) ? (a.max_length - P) : (Ln - P);
    const float best_run = t_run[run_pos[0]] / (float)pow((double)bhl, (double)a.length_penalty);
    float worst = INFINITY;
    int all_fin = 1;
    for (int j = 0; j < nb; ++j) {
      worst = fminf(worst, a.fin_score[(int64_t)b * nb + j]);
      all_fin &= a.fin_flag[(int64_t)b * nb + j] != 0;
    }
    int any_better = 0;
    for (int j = 0; j < nb; ++j) {
      const float wf = a.fin_flag[(int64_t)b * nb + j] ? worst : NEG;
      any_better |= best_run > wf;
    }
    const int uns = a.unsat[b] && any_better;
    a.unsat[b] = uns;
    int all_hit = 1;
    for (int c = 0; c < K; ++c) all_hit &= t_hit[c];
    a.item_flags[3 * b] = uns;
    a.item_flags[3 * b + 1] = all_fin;
    a.item_flags[3 * b + 2] = all_hit;
    __threadfence();
    const int prev = atomicAdd(a.counter, 1);
    last = prev == (int)a.B - 1;
  }
  __syncthreads();
  // 8. the last item: _beam_search_has_unfinished_sequences over the batch, advance cur_len
  if (last && tid == 0) {
    __threadfence();
    int improve = 0, all_fin = 1, all_hit = 1;
    for (int i = 0; i < (int)a.B; ++i) {
      improve |= __hip_atomic_load(a.item_flags + 3 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      all_fin &= __hip_atomic_load(a.item_flags + 3 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      all_hit &= __hip_atomic_load(a.item_flags + 3 * i + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int open = !(all_fin && a.early_stopping == 1);
    const int go = improve && open && !all_hit;
    *a.go = go;
    if (!go) *a.done = 1;
    *a.counter = 0;
    *a.cur_len = L + 1;
    __threadfence();
  }
}

}  // namespace

extern "C" size_t kw_beam_logprobs_workspace(int64_t R) {
  return (size_t)R * BSPLIT * BPART * sizeof(float) + (size_t)R * sizeof(int);
}

extern "C" int kw_beam_logprobs(const kw_beam_logprobs_args* a, kw_stream_t stream) {
  if (!a || !a->logits || !a->suppress_mask || !a->ids || !a->cur_len || !a->cand_val || !a->cand_idx || !a->done ||
      a->R <= 0 || a->V <= 0 || a->k < 1 || a->k > KMAX || (a->n_begin_suppress > 0 && !a->begin_suppress))
    return kw_set_error_msg(KW_EINVAL, "kw_beam_logprobs: invalid arguments (k <= 16)");
  if (a->workspace && a->ws_bytes >= kw_beam_logprobs_workspace(a->R) && a->V <= (int64_t)BSPLIT * BT_S * BUNR)
    hipLaunchKernelGGL(beam_logprobs_split_kernel, dim3((unsigned)a->R, BSPLIT), dim3(BT_S), 0, (hipStream_t)stream, *a);
  else
    hipLaunchKernelGGL(beam_logprobs_kernel, dim3((unsigned)a->R), dim3(ST), 0, (hipStream_t)stream, *a);
  KW_CHECK_LAUNCH();
  return KW_OK;
}

extern "C" int kw_beam_select(const kw_beam_select_args* a, kw_stream_t stream) {
  if (!a || a->B <= 0 || a->num_beams < 2 || a->num_beams > NBMAX || a->V <= 0 || !a->cand_val || !a->cand_idx ||
      !a->ids || !a->run_scores || !a->fin_seq || !a->fin_score || !a->fin_len || !a->fin_flag ||
      !a->unsat || !a->cur_len || !a->counter || !a->go || !a->done || !a->item_flags || a->fin_stride > TMAX ||
      a->ids_stride < a->max_length || a->fin_stride < a->max_length || a->max_length > TMAX ||
      (a->bp && a->bp_stride < a->max_length))
    return kw_set_error_msg(KW_EINVAL, "kw_beam_select: invalid arguments (2 <= num_beams <= 8, max_length <= 512)");
  hipLaunchKernelGGL(beam_select_kernel, dim3((unsigned)a->B), dim3(BT), 0, (hipStream_t)stream, *a);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
