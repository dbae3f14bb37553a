// Whisper logits processors on device, shared by the greedy (sampling.hip) and beam (beam.hip) steps.
// SuppressTokens (TF/generation/logits_process.py:1869-1906) -> SuppressTokensAtBegin (:1816-1866,
// when input_ids.shape[-1] == begin_index) -> WhisperTimeStamp (:1909-2047): the per-row state (last /
// penultimate token, last timestamp, first step) is re-derived from the row's own id history each step,
// exactly as the reference re-derives it from input_ids.
#pragma once
#include <math.h>

#include "kw_common.h"

namespace kwp {

constexpr int ST = 1024;

struct RowState {
  int L, begin, ts_begin, no_ts, eos;
  int rt;          // return_timestamps
  int last_ts, pen_ts, has_stamp, stamp_lo;  // stamp_lo: first allowed timestamp id
  int first_step;
  int max_init;    // -1 = none
  int ban_text;
};

// process() with the SuppressTokens flag of v already loaded: the split kernels fetch the mask bytes of their
// slice together with the logits (a mask load inside the per-element compare chain cost one vmcnt(0) round
// trip per element)
__device__ __forceinline__ float process_m(const RowState& st, bool masked, const int32_t* __restrict__ bsup,
                                           int nbsup, int v, float x) {
  if (masked) return -INFINITY;
  if (st.first_step) {
    for (int i = 0; i < nbsup; ++i)
      if (bsup[i] == v) return -INFINITY;
  }
  if (st.rt) {
    if (v == st.no_ts) return -INFINITY;
    if (st.last_ts) {
      if (st.pen_ts) {
        if (v >= st.ts_begin) return -INFINITY;
      } else {
        if (v < st.eos) return -INFINITY;
      }
    }
    if (st.has_stamp && v >= st.ts_begin && v < st.stamp_lo) return -INFINITY;
    if (st.first_step) {
      if (v < st.ts_begin) return -INFINITY;
      if (st.max_init >= 0 && v > st.ts_begin + st.max_init) return -INFINITY;
    }
    if (st.ban_text && v < st.ts_begin) return -INFINITY;
  }
  return x;
}

__device__ __forceinline__ float process(const RowState& st, const uint8_t* __restrict__ mask,
                                         const int32_t* __restrict__ bsup, int nbsup, int v, float x) {
  return process_m(st, mask[v] != 0, bsup, nbsup, v, x);
}

__device__ float block_reduce_max(float v, float* sh) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < ST / 64; ++i) r = fmaxf(r, sh[i]);
  __syncthreads();
  return r;
}

__device__ float block_reduce_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < ST / 64; ++i) r += sh[i];
  __syncthreads();
  return r;
}


// Per-row processor state from the id history [begin, L) (one 1024-thread workgroup per row).
__device__ __forceinline__ RowState row_state(const int64_t* __restrict__ ids, int L, int begin, int ts_begin,
                                              int no_ts, int eos, int rt, int max_init, int* fin_out,
                                              int (*shi)[2], RowState* st_sh) {
  const int tid = threadIdx.x;
  int fin = 0, last_stamp_pos = -1;
  for (int p = begin + tid; p < L; p += ST) {
    const int64_t t = ids[p];
    if (t == eos) fin = 1;
    if (t >= ts_begin && p > last_stamp_pos) last_stamp_pos = p;
  }
  fin = __syncthreads_or(fin);
  {
    int v = last_stamp_pos;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    if ((tid & 63) == 0) shi[tid >> 6][0] = v;
  }
  __syncthreads();
  if (tid == 0) {
    int lp = shi[0][0];
    for (int i = 1; i < ST / 64; ++i) lp = max(lp, shi[i][0]);
    RowState st;
    st.L = L; st.begin = begin; st.ts_begin = ts_begin; st.no_ts = no_ts; st.eos = eos;
    st.rt = rt; st.max_init = max_init; st.ban_text = 0;
    const int n = L - begin;
    st.first_step = (L == begin);
    st.last_ts = n >= 1 && ids[L - 1] >= ts_begin;
    st.pen_ts = n < 2 || ids[L - 2] >= ts_begin;
    st.has_stamp = lp >= 0;
    if (st.has_stamp) {
      const int last_stamp = (int)ids[lp];
      st.stamp_lo = (st.last_ts && !st.pen_ts) ? last_stamp : last_stamp + 1;
    } else {
      st.stamp_lo = 0;
    }
    *st_sh = st;
  }
  __syncthreads();
  *fin_out = fin;
  return *st_sh;
}

// WhisperTimeStamp's probability-mass rule (logits_process.py:2040-2045) on the processed scores
// s(v) = process(.., f(v)): ban text when logsumexp(logprobs[ts:]) > max(logprobs[:ts]).  Shift
// invariant, so f may be raw logits (greedy) or log-probs (beam).
template <typename F>
__device__ __forceinline__ void timestamp_rule(RowState& st, const uint8_t* mask, const int32_t* bsup, int nbsup,
                                               int V, F f, float* shf) {
  const int tid = threadIdx.x;
  float m_all = -INFINITY, m_text = -INFINITY, m_ts = -INFINITY;
#pragma unroll 8
  for (int v = tid; v < V; v += ST) {
    const float s = process(st, mask, bsup, nbsup, v, f(v));
    m_all = fmaxf(m_all, s);
    if (v < st.ts_begin) m_text = fmaxf(m_text, s); else m_ts = fmaxf(m_ts, s);
  }
  m_all = block_reduce_max(m_all, shf);
  m_text = block_reduce_max(m_text, shf);
  m_ts = block_reduce_max(m_ts, shf);
  float sum = 0.f;
#pragma unroll 8
  for (int v = tid; v < V; v += ST) {
    const float s = process(st, mask, bsup, nbsup, v, f(v));
    sum += expf(s - m_all);
  }
  sum = block_reduce_sum(sum, shf);
  const float lse = logf(sum);
  const float lp_text_max = (m_text - m_all) - lse;
  const float lp_ts_max = (m_ts - m_all) - lse;
  float tsum = 0.f;
  if (lp_ts_max > -INFINITY) {
    for (int v = st.ts_begin + tid; v < V; v += ST) {
      const float s = process(st, mask, bsup, nbsup, v, f(v));
      const float lp = (s - m_all) - lse;
      tsum += expf(lp - lp_ts_max);
    }
  }
  tsum = block_reduce_sum(tsum, shf);
  const float ts_lse = lp_ts_max > -INFINITY ? lp_ts_max + logf(tsum) : -INFINITY;
  if (ts_lse > lp_text_max) st.ban_text = 1;
}

}  // namespace kwp
