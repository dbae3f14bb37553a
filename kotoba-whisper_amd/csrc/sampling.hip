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

}  // namespace

extern "C" int kw_greedy_step(const kw_sampler_args* a, kw_stream_t stream) {
  if (!a || !a->logits || !a->suppress_mask || !a->ids || !a->cur_len || !a->unfinished || !a->counter || !a->n_unfinished || a->B <= 0 ||
      a->V <= 0 || (a->n_begin_suppress > 0 && !a->begin_suppress))
    return kw_set_error_msg(KW_EINVAL, "kw_greedy_step: invalid arguments");
  hipLaunchKernelGGL(greedy_step_kernel, dim3((unsigned)a->B), dim3(ST), 0, (hipStream_t)stream, *a);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
