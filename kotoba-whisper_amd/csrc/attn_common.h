// Decode-attention building blocks shared by the attention kernels (attention.hip) and the fused QKV +
// self-attention step (qkvself.hip): 16-B key/value row registers, the bf16 one-row softmax arithmetic
// (log2-unit scores, per-wave references, merged in wave order) and the {value, tag} granule hand-off.
#pragma once
#include <math.h>

#include "kw_common.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr int HD = 64;  // head_dim of every Whisper model

template <typename T>
struct Row8 {
  u32x4 u[sizeof(T) == 2 ? 1 : 2];
};
template <typename T>
__device__ __forceinline__ Row8<T> ld_row8(const T* p) {  // streamed once per step: non-temporal
  Row8<T> r;
  r.u[0] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  if constexpr (sizeof(T) == 4) r.u[1] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + 1);
  return r;
}
template <typename T>
__device__ __forceinline__ void unpack8(const Row8<T>& r, float v[8]) {
  if constexpr (sizeof(T) == 2) {
    const uint32_t w[4] = {r.u[0][0], r.u[0][1], r.u[0][2], r.u[0][3]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    const uint32_t w[8] = {r.u[0][0], r.u[0][1], r.u[0][2], r.u[0][3], r.u[1][0], r.u[1][1], r.u[1][2], r.u[1][3]};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = __uint_as_float(w[i]);
  }
}

// bf16 decode attention, one query row over one wave's key groups j (lane (slot, sub) holds 16 B of key rows
// slot + 32 j): scores in log2 units (the query carries log2 e, so p = exp2(s - m) is one v_exp), the wave's
// OWN softmax reference m_w (no workgroup barrier between the scores and the values), the row sum and the 8
// value dims of this lane reduced over the wave's key slots.  The workgroup merges its waves' (m_w, l_w, o_w)
// once at the end (merge_waves_bf16), and chunks merge with exp2 of log2-unit maxima.  Every multiply-add is
// an explicit fmaf so every kernel that uses these helpers rounds identically (bitwise-equal rows).
// the two halves of wave_row_bf16, for kernels that interleave loads between them: the scores (log2 units)
// and the wave maximum ...
// JV: the first key group j that can fall past the chunk end (a caller whose chunks all hold more than KS * (JV - 1)
// keys passes JV > 0 and the groups below it skip the check; the arithmetic is the same)
template <int KS = 32, int JV = 0>  // key of (slot, j) = k0 + slot + KS * j (32 key slots per 4-wave row, 16 per 2-wave row)
__device__ __forceinline__ float wave_scores_bf16(const float ql[8], const u32x4 kr[8], int k0, int k1, int slot,
                                                  int nj, float sc[8]) {
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = -INFINITY;
    if (j < nj) {
      const uint32_t w[4] = {kr[j][0], kr[j][1], kr[j][2], kr[j][3]};
      float sj = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sj = fmaf(ql[2 * i], __uint_as_float(w[i] << 16), sj);
        sj = fmaf(ql[2 * i + 1], __uint_as_float(w[i] & 0xffff0000u), sj);
      }
      sj = kw_sum8(sj);
      sc[j] = (j < JV || k0 + slot + KS * j < k1) ? sj : -INFINITY;
      mx = fmaxf(mx, sc[j]);
    }
  }
  return wave_max(mx);
}

// ... then p = exp2(s - m_w), the row sum and this lane's 8 value dims reduced over the wave's key slots
template <int KS = 32, int JV = 0>
__device__ __forceinline__ void wave_values_bf16(const float sc[8], float mx, const u32x4 vr[8], int k0, int k1,
                                                 int slot, int nj, float& lw, float acc[8]) {
  float lsum = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j < nj) {
      const bool valid = j < JV || k0 + slot + KS * j < k1;
      const float pj = valid ? __builtin_amdgcn_exp2f(sc[j] - mx) : 0.f;
      lsum += pj;
      // a masked slot holds a clamped row that may be STALE (a cache row this step has not written yet, e.g. the
      // new position's row before its append): p = 0 times a stale NaN / Inf is NaN, so its values are zeroed
      const uint32_t w[4] = {valid ? vr[j][0] : 0u, valid ? vr[j][1] : 0u, valid ? vr[j][2] : 0u,
                             valid ? vr[j][3] : 0u};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[2 * i] = fmaf(pj, __uint_as_float(w[i] << 16), acc[2 * i]);
        acc[2 * i + 1] = fmaf(pj, __uint_as_float(w[i] & 0xffff0000u), acc[2 * i + 1]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = kw_sum_hi(acc[i]);
  lw = wave_sum_dpp(lsum) * 0.125f;  // every row's p was counted by its 8 lanes (exact: power of two)
}

template <int KS = 32>
__device__ __forceinline__ void wave_row_bf16(const float ql[8], const u32x4 kr[8], const u32x4 vr[8], int k0, int k1,
                                              int slot, int nj, float& mw, float& lw, float acc[8]) {
  float sc[8];
  mw = wave_scores_bf16<KS>(ql, kr, k0, k1, slot, nj, sc);
  wave_values_bf16<KS>(sc, mw, vr, k0, k1, slot, nj, lw, acc);
}

// One wave's running softmax over a pair's chunks, in chunk order: (M, Lr, A) absorbs the chunk's (m_w, l_w,
// acc) -- a wave with no valid key in the chunk (m_w = -inf) is skipped, the first valid chunk is copied, later
// ones merge with exp2 rescales.  fold_begin updates (M, Lr) and returns the mode; fold_value applies it to one
// accumulator.  Shared by cross_attn_row_kernel (a wave folds as it streams) and the chunk-grid kernels' combine
// (the final chunk folds every chunk's published wave partials), so the two are bitwise equal.
__device__ __forceinline__ int fold_begin(float mw, float lw, float& M, float& Lr, float& f0, float& f1) {
  if (mw == -INFINITY) return 0;
  if (M == -INFINITY) {
    M = mw;
    Lr = lw;
    return 1;
  }
  const float mn = fmaxf(M, mw);
  f0 = __builtin_amdgcn_exp2f(M - mn);
  f1 = __builtin_amdgcn_exp2f(mw - mn);
  Lr = fmaf(Lr, f0, lw * f1);
  M = mn;
  return 2;
}
__device__ __forceinline__ float fold_value(int mode, float A, float acc, float f0, float f1) {
  return mode == 0 ? A : mode == 1 ? acc : fmaf(A, f0, acc * f1);
}

// a workgroup's 4 waves: (m_w, l_w) at st[w], st[4 + w]; o_w at rd[w][dim] -> the chunk's (m, l, o[dim])
__device__ __forceinline__ void merge_waves_bf16(const float* st, const float (*rd)[64], int dim, float& m, float& l,
                                                 float& o) {
  m = fmaxf(fmaxf(st[0], st[1]), fmaxf(st[2], st[3]));
  float f[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) f[w] = __builtin_amdgcn_exp2f(st[w] - m);  // a wave with no valid key: m_w -inf -> 0
  l = fmaf(st[4], f[0], st[5] * f[1]) + fmaf(st[6], f[2], st[7] * f[3]);
  o = dim < HD ? fmaf(rd[0][dim], f[0], rd[1][dim] * f[1]) + fmaf(rd[2][dim], f[2], rd[3][dim] * f[3]) : 0.f;
}

// exp of a chunk maximum's offset: log2 units for bf16 rows (wave_row_bf16), natural units for f32
template <typename T>
__device__ __forceinline__ float chunk_scale(float d) {
  if constexpr (sizeof(T) == 2) return __builtin_amdgcn_exp2f(d);
  else return expf(d);
}

constexpr int XG_SPIN_LIMIT = 1 << 22;

__device__ __forceinline__ void put_granule(unsigned long long* g, float v) {
  __hip_atomic_store(g, (1ull << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long peek_granule(const unsigned long long* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace
