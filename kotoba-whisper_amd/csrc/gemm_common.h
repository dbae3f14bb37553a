// Shared GEMM parameter block and epilogue (gemm.hip).
#pragma once
#include "kw_common.h"

namespace kwg {

struct GemmP {
  const void* A;
  int64_t lda, a_rpb, a_bs;
  const void* W;
  const float* bias;
  void* C;
  int64_t ldc, c_rpb, c_bs;
  int M, N, K;
  int gelu;
  float scale;
  int scale_cols;
  const float* row_add;
  int row_add_period;
  int hs_seq, hs_heads, hs_hd;
};

__device__ __forceinline__ int64_t row_off(int64_t r, int64_t rpb, int64_t bs, int64_t ld) {
  const int64_t b = r / rpb;
  return b * bs + (r - b * rpb) * ld;
}

template <int EPI, typename TC>
__device__ __forceinline__ void epi_one(const GemmP& p, int m, int n, float v, float bias_n) {
  v += bias_n;
  if constexpr (EPI == KW_EPI_RESID) {
    float* c = reinterpret_cast<float*>(p.C) + row_off(m, p.c_rpb, p.c_bs, p.ldc) + n;
    *c += v;
  } else {
    if (p.gelu) v = gelu_erf(v);
    if (n < p.scale_cols) v *= p.scale;
    if (p.row_add) v += p.row_add[(int64_t)(m % p.row_add_period) * p.N + n];
    int64_t off;
    if constexpr (EPI == KW_EPI_HEADSPLIT) {
      const int width = p.hs_heads * p.hs_hd;
      const int part = n / width;
      const int rem = n - part * width;
      const int h = rem / p.hs_hd, d = rem - h * p.hs_hd;
      const int b = m / p.hs_seq, t = m - b * p.hs_seq;
      const int nb = p.M / p.hs_seq;
      off = ((((int64_t)part * nb + b) * p.hs_heads + h) * p.hs_seq + t) * p.hs_hd + d;
    } else {
      off = row_off(m, p.c_rpb, p.c_bs, p.ldc) + n;
    }
    TypeIO<TC>::st(reinterpret_cast<TC*>(p.C) + off, v);
  }
}

inline GemmP to_params(const kw_gemm_args* a) {
  GemmP p;
  p.A = a->A; p.lda = a->lda;
  p.a_rpb = a->a_rows_per_batch > 0 ? a->a_rows_per_batch : a->M;
  p.a_bs = a->a_batch_stride;
  p.W = a->W; p.bias = a->bias; p.C = a->C; p.ldc = a->ldc;
  p.c_rpb = a->c_rows_per_batch > 0 ? a->c_rows_per_batch : a->M;
  p.c_bs = a->c_batch_stride;
  p.M = (int)a->M; p.N = (int)a->N; p.K = (int)a->K;
  p.gelu = a->gelu; p.scale = a->scale; p.scale_cols = (int)a->scale_cols;
  p.row_add = a->row_add; p.row_add_period = a->row_add_period > 0 ? (int)a->row_add_period : 1;
  p.hs_seq = a->hs_seq > 0 ? (int)a->hs_seq : 1; p.hs_heads = a->hs_heads > 0 ? (int)a->hs_heads : 1;
  p.hs_hd = a->hs_head_dim > 0 ? (int)a->hs_head_dim : 1;
  if (p.c_rpb <= 0) p.c_rpb = 1;
  if (p.a_rpb <= 0) p.a_rpb = 1;
  return p;
}

inline int check_common(const kw_gemm_args* a) {
  if (!a || !a->A || !a->W || !a->C || a->M < 0 || a->N <= 0 || a->K <= 0)
    return kw_set_error_msg(KW_EINVAL, "kw_gemm: null pointer or bad sizes");
  if (a->epilogue == KW_EPI_RESID && a->c_dtype != KW_DT_F32)
    return kw_set_error_msg(KW_EINVAL, "kw_gemm: RESID epilogue needs an f32 C");
  if (a->epilogue == KW_EPI_HEADSPLIT && (a->hs_seq <= 0 || a->hs_heads <= 0 || a->hs_head_dim <= 0 ||
                                          a->M % a->hs_seq != 0 || a->N % (a->hs_heads * a->hs_head_dim) != 0))
    return kw_set_error_msg(KW_EINVAL, "kw_gemm: bad head-split geometry");
  if (a->epilogue < 0 || a->epilogue > 2) return kw_set_error_msg(KW_EINVAL, "kw_gemm: bad epilogue");
  return KW_OK;
}

}  // namespace kwg
