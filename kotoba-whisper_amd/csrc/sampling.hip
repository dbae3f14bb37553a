// Greedy decode step on device (K14 + K15): logits processors, argmax, finished-row handling and
// the cur_len advance -- no host sync per step, so a whole decode step can live in one hipGraph.
//
// Reference order (transformers 5.15.0): SuppressTokens (TF/generation/logits_process.py:1869-1906)
// -> SuppressTokensAtBegin (:1816-1866, when input_ids.shape[-1] == begin_index) -> WhisperTimeStamp
// (:1909-2047, only with return_timestamps) -> argmax (TF/generation/utils.py:2925, first max wins)
// -> finished rows emit pad (:2929) -> MaxLength / EOS stopping (stopping_criteria.py:75-77).
// The WhisperTimeStamp per-row state (last / penultimate token, last timestamp, finished flag) is
// derived from the row's own id history each step, exactly as the reference re-derives it from
// input_ids.  One 1024-thread workgroup per row; the processed row is recomputed on the fly in each
// of the four L2-resident passes (max, sum, timestamp log-sum-exp, argmax) instead of materialised.
#include <math.h>

#include "kw_common.h"

namespace {

constexpr int ST = 1024;

struct RowState {
  int L, begin, ts_begin, no_ts, eos;
  int rt;          // return_timestamps
  int last_ts, pen_ts, has_stamp, stamp_lo;  // stamp_lo: first allowed timestamp id
  int first_step;
  int max_init;    // -1 = none
  int ban_text;
};

__device__ __forceinline__ float process(const RowState& st, const uint8_t* __restrict__ mask,
                                         const int32_t* __restrict__ bsup, int nbsup, int v, float x) {
  if (mask[v]) return -INFINITY;
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

__global__ __launch_bounds__(ST) void greedy_step_kernel(kw_sampler_args a) {
  __shared__ float shf[ST / 64];
  __shared__ int shi[ST / 64][2];
  __shared__ RowState st_sh;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int L = *a.cur_len;
  const int64_t* ids = a.ids + (int64_t)b * a.ids_stride;
  const float* x = a.logits + (int64_t)b * a.V;
  const int V = (int)a.V;

  // ---- history scan: finished flag and last timestamp position ---------------------------------
  int fin = 0, last_stamp_pos = -1;
  for (int p = a.begin_index + tid; p < L; p += ST) {
    const int64_t t = ids[p];
    if (t == a.eos_id) fin = 1;
    if (t >= a.ts_begin && p > last_stamp_pos) last_stamp_pos = p;
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
    st.L = L; st.begin = a.begin_index; st.ts_begin = a.ts_begin; st.no_ts = a.no_ts_id; st.eos = a.eos_id;
    st.rt = a.return_timestamps; st.max_init = a.max_initial_ts; st.ban_text = 0;
    const int n = L - a.begin_index;
    st.first_step = (L == a.begin_index);
    st.last_ts = n >= 1 && ids[L - 1] >= a.ts_begin;
    st.pen_ts = n < 2 || ids[L - 2] >= a.ts_begin;
    st.has_stamp = lp >= 0;
    if (st.has_stamp) {
      const int last_stamp = (int)ids[lp];
      st.stamp_lo = (st.last_ts && !st.pen_ts) ? last_stamp : last_stamp + 1;
    } else {
      st.stamp_lo = 0;
    }
    st_sh = st;
  }
  __syncthreads();
  RowState st = st_sh;

  // ---- timestamp probability-mass rule (logits_process.py:2040-2045) ---------------------------
  if (st.rt) {
    float m_all = -INFINITY, m_text = -INFINITY, m_ts = -INFINITY;
    for (int v = tid; v < V; v += ST) {
      const float s = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, x[v]);
      m_all = fmaxf(m_all, s);
      if (v < st.ts_begin) m_text = fmaxf(m_text, s); else m_ts = fmaxf(m_ts, s);
    }
    m_all = block_reduce_max(m_all, shf);
    m_text = block_reduce_max(m_text, shf);
    m_ts = block_reduce_max(m_ts, shf);
    float sum = 0.f;
    for (int v = tid; v < V; v += ST) {
      const float s = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, x[v]);
      sum += expf(s - m_all);
    }
    sum = block_reduce_sum(sum, shf);
    const float lse = logf(sum);
    // logprobs = (s - max) - log(sum); compare logsumexp(logprobs[ts:]) with max(logprobs[:ts])
    const float lp_text_max = (m_text - m_all) - lse;
    const float lp_ts_max = (m_ts - m_all) - lse;
    float tsum = 0.f;
    if (lp_ts_max > -INFINITY) {
      for (int v = st.ts_begin + tid; v < V; v += ST) {
        const float s = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, x[v]);
        const float lp = (s - m_all) - lse;
        tsum += expf(lp - lp_ts_max);
      }
    }
    tsum = block_reduce_sum(tsum, shf);
    const float ts_lse = lp_ts_max > -INFINITY ? lp_ts_max + logf(tsum) : -INFINITY;
    if (ts_lse > lp_text_max) st.ban_text = 1;
  }

  // ---- argmax (first index on ties) -----------------------------------------------------------
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = tid; v < V; v += ST) {
    const float s = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, x[v]);
    if (a.scores_out) a.scores_out[(int64_t)b * a.V + v] = s;
    if (s > best || (s == best && v < bi)) { best = s; bi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if ((tid & 63) == 0) { shf[tid >> 6] = best; shi[tid >> 6][1] = bi; }
  __syncthreads();
  if (tid == 0) {
    float bb = shf[0];
    int ii = shi[0][1];
    for (int i = 1; i < ST / 64; ++i) {
      if (shf[i] > bb || (shf[i] == bb && shi[i][1] < ii)) { bb = shf[i]; ii = shi[i][1]; }
    }
    if (ii == 0x7fffffff) ii = 0;  // all -inf (cannot happen with a sane config): torch.argmax -> 0
    const int64_t tok = fin ? (int64_t)a.pad_id : (int64_t)ii;
    a.ids[(int64_t)b * a.ids_stride + L] = tok;
    const int done = fin || tok == a.eos_id || (L + 1) >= a.max_length;
    a.unfinished[b] = done ? 0 : 1;
    __threadfence();
    const int prev = atomicAdd(a.counter, 1);
    if (prev == (int)a.B - 1) {
      __threadfence();
      int n = 0;
      for (int i = 0; i < (int)a.B; ++i) n += __hip_atomic_load(a.unfinished + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *a.n_unfinished = n;
      *a.counter = 0;
      *a.cur_len = L + 1;
      __threadfence();
    }
  }
}

}  // namespace

extern "C" int kw_greedy_step(const kw_sampler_args* a, kw_stream_t stream) {
  if (!a || !a->logits || !a->suppress_mask || !a->ids || !a->cur_len || !a->unfinished || !a->counter || !a->n_unfinished || a->B <= 0 ||
      a->V <= 0 || (a->n_begin_suppress > 0 && !a->begin_suppress))
    return kw_set_error_msg(KW_EINVAL, "kw_greedy_step: invalid arguments");
  hipLaunchKernelGGL(greedy_step_kernel, dim3((unsigned)a->B), dim3(ST), 0, (hipStream_t)stream, *a);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
