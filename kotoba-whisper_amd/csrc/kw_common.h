// Shared helpers for the kwhisper CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/kwhisper.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef uint16_t bf16_t;  // storage type for bf16 in global memory

#define KW_WAVE 64

#ifndef KW_POLL_SLEEP
#define KW_POLL_SLEEP 1  // s_sleep units (64 cycles) between the polls of an in-launch hand-off
#endif

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  // round-to-nearest-even; NaN stays NaN (plain cast lowers to v_cvt_pk_bf16_f32 on gfx950)
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<bf16_t*>(&b);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  // two RNE conversions in one v_cvt_pk_bf16_f32; lo in bits 0-15
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

template <typename T> struct TypeIO;
template <> struct TypeIO<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <> struct TypeIO<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
};

__device__ __forceinline__ float gelu_erf(float x) {
  // exact GELU (TF/activations.py:70-89, nn.functional.gelu default)
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

__device__ __forceinline__ float gelu_bf16out(float x) {
  // GELU for a bf16 result: erf by Abramowitz & Stegun 7.1.26 (|err| <= 1.5e-7, far below bf16's
  // 2^-9 rounding) -- one rcp + one exp instead of the erff library call; f32 results use gelu_erf
  // 0.5 x (1 + sign(x) e) = h + |h| e with h = x / 2; erf(|x|/sqrt2) = e = 1 - poly(t) exp(-x^2/2)
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752440f, fabsf(x), 1.0f));
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float e = fmaf(-poly, __builtin_amdgcn_exp2f(x * x * -0.72134752044448170368f), 1.0f);  // -log2(e)/2
  const float h = 0.5f * x;
  return fmaf(fabsf(h), e, h);
}

// Cross-lane reductions on the VALU (DPP within 16-lane rows, v_permlane16/32_swap across them) instead of
// ds_bpermute round trips through the LDS unit.  Every step combines a lane with exactly the partner of the
// xor butterfly it replaces (quad_perm [1,0,3,2] = ^1, [2,3,0,1] = ^2; once 4- / 8-lane groups are uniform,
// row_half_mirror / row_mirror pair them like ^4 / ^8; row_ror:8 = ^8; the swaps = ^16 / ^32) and + / max
// are commutative, so results are bitwise those of the __shfl_xor butterflies they replace (max in any order).
// The lanes a step reads must be active.
template <int CTRL>
__device__ __forceinline__ float kw_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float kw_swap16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float kw_swap32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float kw_swap16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float kw_swap32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// sum over each aligned 8-lane group (lane bits 0..2): the ^1, ^2, ^4 butterfly
__device__ __forceinline__ float kw_sum8(float v) {
  v += kw_dpp<0xB1>(v);
  v += kw_dpp<0x4E>(v);
  return v + kw_dpp<0x141>(v);
}
// sum over lane bits 3..5 (lanes with equal l & 7): the ^8, ^16, ^32 butterfly
__device__ __forceinline__ float kw_sum_hi(float v) {
  v += kw_dpp<0x128>(v);
  return kw_swap32_sum(kw_swap16_sum(v));
}
// (keeps the ^32 .. ^1 order of the original butterfly: a different association tree would change f32 sums)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// the same butterfly on DPP / permlane (no LDS round trips); a different association than wave_sum
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += kw_dpp<0xB1>(v);
  v += kw_dpp<0x4E>(v);
  v += kw_dpp<0x141>(v);
  v += kw_dpp<0x140>(v);
  return kw_swap32_sum(kw_swap16_sum(v));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, kw_dpp<0xB1>(v));
  v = fmaxf(v, kw_dpp<0x4E>(v));
  v = fmaxf(v, kw_dpp<0x141>(v));
  v = fmaxf(v, kw_dpp<0x140>(v));
  return kw_swap32_max(kw_swap16_max(v));
}

#define KW_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return kw_set_error(_e);          \
  } while (0)

int kw_set_error(hipError_t e);
int kw_set_error_msg(int code, const char* msg);
