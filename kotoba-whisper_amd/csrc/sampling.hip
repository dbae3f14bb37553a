// Greedy decode step on device (K14 + K15): logits processors, argmax, finished-row handling and
// the cur_len advance -- no host sync per step, so a whole decode step can live in one hipGraph.
//
// Reference order (transformers 5.15.0): SuppressTokens (TF/generation/logits_process.py:1869-1906)
// -> SuppressTokensAtBegin (:1816-1866, when input_ids.shape[-1] == begin_index) -> WhisperTimeStamp
// (:1909-2047, only with return_timestamps) -> argmax (TF/generation/utils.py:2925, first max wins)
// -> finished rows emit pad (:2929) -> MaxLength / EOS stopping (stopping_criteria.py:75-77).
// The WhisperTimeStamp per-row state (last / penultimate token, last timestamp, finished flag) is
// derived from the row's own id history each step, exactly as the reference re-derives it from
// input_ids.  With timestamps: one 1024-thread workgroup per row; the processed row is recomputed on
// the fly in each of the four L2-resident passes (max, sum, timestamp log-sum-exp, argmax) instead of
// materialised.  Without: greedy_step_split_kernel (a row over NSPLIT workgroups).
#include <math.h>

#include "processors.h"

namespace {

using namespace kwp;

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

  // ---- history: finished flag and the WhisperTimeStamp row state --------------------------------
  int fin = 0;
  RowState st = row_state(ids, L, a.begin_index, a.ts_begin, a.no_ts_id, a.eos_id, a.return_timestamps,
                          a.max_initial_ts, &fin, shi, &st_sh);
  // ---- timestamp probability-mass rule (logits_process.py:2040-2045) ---------------------------
  if (st.rt) timestamp_rule(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, V, [&](int v) { return x[v]; }, shf);

  // ---- argmax (first index on ties) -----------------------------------------------------------
  // 8 loads of the logits and the suppress mask in flight per thread before any compare (a one-load
  // loop pays an L2 round trip per 4 KB of the row)
  float best = -INFINITY;
  int bi = 0x7fffffff;
  constexpr int UNR = 8;
  for (int v0 = tid; v0 < V; v0 += ST * UNR) {
    float xv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int v = v0 + u * ST;
      xv[u] = v < V ? x[v] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int v = v0 + u * ST;
      if (v < V) {
        const float s = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, xv[u]);
        if (a.scores_out) a.scores_out[(int64_t)b * a.V + v] = s;
        if (s > best || (s == best && v < bi)) { best = s; bi = v; }
      }
    }
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

// Split-row variant (no timestamps, no scores_out): row b's V logits are cut into NSPLIT slices of one
// 512-thread workgroup each (16 loads in flight per thread: one memory round trip per slice instead of
// a serial walk over the row); each slice publishes its (max, first index, finished flag) write-through,
// and the last of all B x NSPLIT workgroups to arrive combines every row's slices in slice order (first
// index on ties, as torch.argmax) and finishes the step exactly as greedy_step_kernel does.
constexpr int SPLIT_T = 512, NSPLIT = 8, SUNR = 16, PART = 8;  // PART: floats published per slice

__global__ __launch_bounds__(SPLIT_T) void greedy_step_split_kernel(kw_sampler_args a) {
  __shared__ float shf[SPLIT_T / 64];
  __shared__ int shi[SPLIT_T / 64];
  const int b = blockIdx.x, sl = blockIdx.y;
  const int tid = threadIdx.x;
  const int L = *a.cur_len;
  const int64_t* ids = a.ids + (int64_t)b * a.ids_stride;
  const float* x = a.logits + (int64_t)b * a.V;
  const int V = (int)a.V;
  const int per = (V + NSPLIT - 1) / NSPLIT;
  const int v0 = sl * per, v1 = min(V, v0 + per);
  const bool first = L == a.begin_index;
  // the slice's logits and SuppressTokens bytes all in flight first (a mask load inside the compare chain
  // below cost one round trip per element; the history scan's loop waits on every load it has issued)
  float xv[SUNR];
  bool mk[SUNR];
#pragma unroll
  for (int u = 0; u < SUNR; ++u) {
    const int v = v0 + tid + u * SPLIT_T, vc = min(v, v1 - 1);  // unconditional (clamped) loads: no branches
    const float xr = x[vc];                                           // and phis between them
    const uint8_t mr = a.suppress_mask[vc];
    xv[u] = v < v1 ? xr : -INFINITY;
    mk[u] = v < v1 ? mr != 0 : true;
  }
  // a row is finished once it emitted EOS (stopping_criteria.py:75-77): one id per thread, in parallel
  // (the row's last arriver needs it; a serial walk there would pay one load latency per position)
  int fin = 0;
  for (int p = a.begin_index + tid; p < L; p += SPLIT_T) fin |= ids[p] == a.eos_id;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int vb = v0; vb < v1; vb += SPLIT_T * SUNR) {  // one round for V <= NSPLIT * 8192
    if (vb != v0) {
#pragma unroll
      for (int u = 0; u < SUNR; ++u) {
        const int v = vb + tid + u * SPLIT_T, vc = min(v, v1 - 1);  // unconditional (clamped) loads: no branches
        const float xr = x[vc];                                           // and phis between them
        const uint8_t mr = a.suppress_mask[vc];
        xv[u] = v < v1 ? xr : -INFINITY;
        mk[u] = v < v1 ? mr != 0 : true;
      }
    }
#pragma unroll
    for (int u = 0; u < SUNR; ++u) {
      const int v = vb + tid + u * SPLIT_T;
      if (v < v1) {
        float s = mk[u] ? -INFINITY : xv[u];
        if (first)
          for (int i = 0; i < a.n_begin_suppress; ++i)
            if (a.begin_suppress[i] == v) s = -INFINITY;
        if (s > best || (s == best && v < bi)) { best = s; bi = v; }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if ((tid & 63) == 0) { shf[tid >> 6] = best; shi[tid >> 6] = bi; }
  fin = __syncthreads_or(fin);
  // one arrival count over all B x NSPLIT workgroups: the last to arrive finishes every row (a thread per
  // row), so the step pays one atomic round trip instead of a per-row count, an ids store + fence and a
  // second count, and the unfinished flags are summed in LDS instead of re-read
  __shared__ int last_sh, nunf_sh;
  if (tid == 0) {
    nunf_sh = 0;
    for (int i = 1; i < SPLIT_T / 64; ++i)
      if (shf[i] > best || (shf[i] == best && shi[i] < bi)) { best = shf[i]; bi = shi[i]; }
    float* part = reinterpret_cast<float*>(a.workspace) + ((int64_t)b * NSPLIT + sl) * PART;
    __hip_atomic_store(part, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<int*>(part) + 1, bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<int*>(part) + 2, fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(a.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_sh = prev == (int)a.B * NSPLIT - 1;
  }
  __syncthreads();
  if (!last_sh) return;
  int n_unf = 0;
  for (int r = tid; r < (int)a.B; r += SPLIT_T) {
    const float* row = reinterpret_cast<const float*>(a.workspace) + (int64_t)r * NSPLIT * PART;
    float pv[NSPLIT];
    int pi[NSPLIT], pf[NSPLIT];
#pragma unroll
    for (int q = 0; q < NSPLIT; ++q) {  // every partial load in flight before the first compare
      pv[q] = __hip_atomic_load(row + PART * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pi[q] = __hip_atomic_load(reinterpret_cast<const int*>(row) + PART * q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pf[q] = __hip_atomic_load(reinterpret_cast<const int*>(row) + PART * q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    float bb = -INFINITY;
    int ii = 0x7fffffff, rf = 0;
#pragma unroll
    for (int q = 0; q < NSPLIT; ++q) {  // slice order = index order: strict > keeps the first max
      if (pv[q] > bb || (pv[q] == bb && pi[q] < ii)) { bb = pv[q]; ii = pi[q]; }
      rf |= pf[q];  // (every slice scanned the same history: all equal)
    }
    if (ii == 0x7fffffff) ii = 0;
    const int64_t tok = rf ? (int64_t)a.pad_id : (int64_t)ii;
    a.ids[(int64_t)r * a.ids_stride + L] = tok;
    const int done = rf || tok == a.eos_id || (L + 1) >= a.max_length;
    a.unfinished[r] = done ? 0 : 1;
    n_unf += done ? 0 : 1;
  }
  if (n_unf) atomicAdd(&nunf_sh, n_unf);
  __syncthreads();
  if (tid == 0) {
    *a.n_unfinished = nunf_sh;
    *a.counter = 0;
    *a.cur_len = L + 1;
  }
}

// Split-row variant WITH timestamps.  WhisperTimeStamp's probability-mass rule (logits_process.py:
// 2040-2045: ban text when logsumexp(logprobs[ts:]) > max(logprobs[:ts])) needs whole-row statistics, so
// each slice publishes, over its processed scores, the text maximum (+ first index), the timestamp
// maximum (+ first index), its own maximum with the sum of exp(s - that maximum), and the timestamp
// sum of exp(s - timestamp maximum); the row's last arriver merges them (log-sum-exp rescaling), applies
// the rule and picks the token (first index on ties, text before timestamps).
__device__ __forceinline__ float blk_max(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < SPLIT_T / 64; ++i) r = fmaxf(r, sh[i]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ float blk_sum(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < SPLIT_T / 64; ++i) r += sh[i];
  __syncthreads();
  return r;
}
__device__ __forceinline__ void blk_argmax(float& best, int& bi, float* shf, int* shi) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if ((threadIdx.x & 63) == 0) { shf[threadIdx.x >> 6] = best; shi[threadIdx.x >> 6] = bi; }
  __syncthreads();
  best = shf[0];
  bi = shi[0];
  for (int i = 1; i < SPLIT_T / 64; ++i)
    if (shf[i] > best || (shf[i] == best && shi[i] < bi)) { best = shf[i]; bi = shi[i]; }
  __syncthreads();
}

__global__ __launch_bounds__(SPLIT_T) void greedy_step_split_ts_kernel(kw_sampler_args a) {
  __shared__ float shf[SPLIT_T / 64];
  __shared__ int shi[SPLIT_T / 64];
  __shared__ RowState st_sh;
  const int b = blockIdx.x, sl = blockIdx.y;
  const int tid = threadIdx.x;
  const int L = *a.cur_len;
  const int64_t* ids = a.ids + (int64_t)b * a.ids_stride;
  const float* x = a.logits + (int64_t)b * a.V;
  const int V = (int)a.V;
  const int per = (V + NSPLIT - 1) / NSPLIT;
  const int v0 = sl * per, v1 = min(V, v0 + per);
  float xv[SUNR];
  bool mk[SUNR];
#pragma unroll
  for (int u = 0; u < SUNR; ++u) {  // the slice's logits and mask bytes in flight while the history is scanned
    const int v = v0 + tid + u * SPLIT_T, vc = min(v, v1 - 1);  // unconditional (clamped) loads: no branches
    const float xr = x[vc];                                           // and phis between them
    const uint8_t mr = a.suppress_mask[vc];
    xv[u] = v < v1 ? xr : -INFINITY;
    mk[u] = v < v1 ? mr != 0 : true;
  }
  // ---- row state from the id history (as kwp::row_state, 512 threads) ----
  int fin = 0, lsp = -1;
  for (int p = a.begin_index + tid; p < L; p += SPLIT_T) {
    const int64_t t = ids[p];
    fin |= t == a.eos_id;
    if (t >= a.ts_begin) lsp = max(lsp, p);
  }
  fin = __syncthreads_or(fin);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lsp = max(lsp, __shfl_xor(lsp, o, 64));
  if ((tid & 63) == 0) shi[tid >> 6] = lsp;
  __syncthreads();
  if (tid == 0) {
    int lp = shi[0];
    for (int i = 1; i < SPLIT_T / 64; ++i) lp = max(lp, shi[i]);
    RowState st;
    st.L = L; st.begin = a.begin_index; st.ts_begin = a.ts_begin; st.no_ts = a.no_ts_id; st.eos = a.eos_id;
    st.rt = 1; st.max_init = a.max_initial_ts; st.ban_text = 0;
    const int n = L - a.begin_index;
    st.first_step = (L == a.begin_index);
    st.last_ts = n >= 1 && ids[L - 1] >= a.ts_begin;
    st.pen_ts = n < 2 || ids[L - 2] >= a.ts_begin;
    st.has_stamp = lp >= 0;
    st.stamp_lo = st.has_stamp ? ((st.last_ts && !st.pen_ts) ? (int)ids[lp] : (int)ids[lp] + 1) : 0;
    st_sh = st;
  }
  __syncthreads();
  const RowState st = st_sh;
  // ---- processed scores of the slice (held in registers) and their statistics ----
  float sv[SUNR];
  float mt = -INFINITY, ms = -INFINITY;
  int it = 0x7fffffff, is = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < SUNR; ++u) {
    const int v = v0 + tid + u * SPLIT_T;
    sv[u] = v < v1 ? process_m(st, mk[u], a.begin_suppress, a.n_begin_suppress, v, xv[u]) : -INFINITY;
    if (v < v1) {
      if (v < st.ts_begin) {
        if (sv[u] > mt || (sv[u] == mt && v < it)) { mt = sv[u]; it = v; }
      } else {
        if (sv[u] > ms || (sv[u] == ms && v < is)) { ms = sv[u]; is = v; }
      }
    }
  }
  for (int vb = v0 + SPLIT_T * SUNR; vb < v1; vb += SPLIT_T) {  // V > NSPLIT * 8192 only
    const int v = vb + tid;
    if (v < v1) {
      const float s = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, x[v]);
      if (v < st.ts_begin) {
        if (s > mt || (s == mt && v < it)) { mt = s; it = v; }
      } else if (s > ms || (s == ms && v < is)) { ms = s; is = v; }
    }
  }
  blk_argmax(mt, it, shf, shi);
  blk_argmax(ms, is, shf, shi);
  const float mall = fmaxf(mt, ms);
  float sa = 0.f, sts = 0.f;
  if (mall > -INFINITY) {
#pragma unroll
    for (int u = 0; u < SUNR; ++u) {
      const int v = v0 + tid + u * SPLIT_T;
      if (v < v1 && sv[u] > -INFINITY) {
        sa += expf(sv[u] - mall);
        if (v >= st.ts_begin) sts += expf(sv[u] - ms);
      }
    }
    for (int vb = v0 + SPLIT_T * SUNR; vb < v1; vb += SPLIT_T) {
      const int v = vb + tid;
      if (v < v1) {
        const float s = process(st, a.suppress_mask, a.begin_suppress, a.n_begin_suppress, v, x[v]);
        if (s > -INFINITY) {
          sa += expf(s - mall);
          if (v >= st.ts_begin) sts += expf(s - ms);
        }
      }
    }
  }
  sa = blk_sum(sa, shf);
  sts = blk_sum(sts, shf);
  if (tid != 0) return;
  float* part = reinterpret_cast<float*>(a.workspace) + ((int64_t)b * NSPLIT + sl) * PART;
  int* rcnt = reinterpret_cast<int*>(a.workspace) + (int64_t)a.B * NSPLIT * PART + b;
  const float vals[7] = {mt, __int_as_float(it), ms, __int_as_float(is), mall, sa, sts};
#pragma unroll
  for (int i = 0; i < 7; ++i) __hip_atomic_store(part + i, vals[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int prev = __hip_atomic_fetch_add(rcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (prev != NSPLIT - 1) return;
  __hip_atomic_store(rcnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float* row = reinterpret_cast<const float*>(a.workspace) + (int64_t)b * NSPLIT * PART;
  float P[NSPLIT][7];
#pragma unroll
  for (int q = 0; q < NSPLIT; ++q)  // every partial load in flight before the merge
#pragma unroll
    for (int i = 0; i < 7; ++i) P[q][i] = __hip_atomic_load(row + PART * q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float bt = -INFINITY, bs = -INFINITY, M = -INFINITY, Mts = -INFINITY;
  int jt = 0x7fffffff, js = 0x7fffffff;
  for (int q = 0; q < NSPLIT; ++q) {  // slice order = index order
    const int qt = __float_as_int(P[q][1]), qs = __float_as_int(P[q][3]);
    if (P[q][0] > bt || (P[q][0] == bt && qt < jt)) { bt = P[q][0]; jt = qt; }
    if (P[q][2] > bs || (P[q][2] == bs && qs < js)) { bs = P[q][2]; js = qs; }
    M = fmaxf(M, P[q][4]);
  }
  Mts = bs;
  float S = 0.f, Sts = 0.f;
  for (int q = 0; q < NSPLIT; ++q) {
    if (P[q][4] > -INFINITY) S += P[q][5] * expf(P[q][4] - M);
    if (P[q][2] > -INFINITY) Sts += P[q][6] * expf(P[q][2] - Mts);
  }
  int ban = 0;
  if (M > -INFINITY) {
    const float lse = logf(S);
    const float lp_text_max = (bt - M) - lse;
    const float lp_ts_max = (Mts - M) - lse;
    const float ts_lse = lp_ts_max > -INFINITY ? lp_ts_max + logf(Sts) : -INFINITY;
    ban = ts_lse > lp_text_max;
  }
  int ii;
  if (ban) ii = js;
  else ii = (bs > bt) ? js : jt;  // a tie keeps the text token (the lower index)
  if (ii == 0x7fffffff) ii = 0;
  const int64_t tok = fin ? (int64_t)a.pad_id : (int64_t)ii;
  a.ids[(int64_t)b * a.ids_stride + L] = tok;
  const int done = fin || tok == a.eos_id || (L + 1) >= a.max_length;
  a.unfinished[b] = done ? 0 : 1;
  __threadfence();
  const int prev2 = atomicAdd(a.counter, 1);
  if (prev2 == (int)a.B - 1) {
    __threadfence();
    int n = 0;
    for (int i = 0; i < (int)a.B; ++i) n += __hip_atomic_load(a.unfinished + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *a.n_unfinished = n;
    *a.counter = 0;
    *a.cur_len = L + 1;
    __threadfence();
  }
}

}  // namespace

extern "C" size_t kw_greedy_step_workspace(int64_t B) {
  return (size_t)B * NSPLIT * PART * sizeof(float) + (size_t)B * sizeof(int);
}

extern "C" int kw_greedy_step(const kw_sampler_args* a, kw_stream_t stream) {
  if (!a || !a->logits || !a->suppress_mask || !a->ids || !a->cur_len || !a->unfinished || !a->counter || !a->n_unfinished || a->B <= 0 ||
      a->V <= 0 || (a->n_begin_suppress > 0 && !a->begin_suppress))
    return kw_set_error_msg(KW_EINVAL, "kw_greedy_step: invalid arguments");
  const bool split = a->workspace && a->ws_bytes >= kw_greedy_step_workspace(a->B) && !a->scores_out;
  if (split && a->return_timestamps)
    hipLaunchKernelGGL(greedy_step_split_ts_kernel, dim3((unsigned)a->B, NSPLIT), dim3(SPLIT_T), 0, (hipStream_t)stream, *a);
  else if (split)
    hipLaunchKernelGGL(greedy_step_split_kernel, dim3((unsigned)a->B, NSPLIT), dim3(SPLIT_T), 0, (hipStream_t)stream, *a);
  else
    hipLaunchKernelGGL(greedy_step_kernel, dim3((unsigned)a->B), dim3(ST), 0, (hipStream_t)stream, *a);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
