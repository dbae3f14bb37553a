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
typedef uint16_t bf16_t;  // storage type for bf16 in global memory

#define KW_WAVE 64

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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

#define KW_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return kw_set_error(_e);          \
  } while (0)

int kw_set_error(hipError_t e);
int kw_set_error_msg(int code, const char* msg);
