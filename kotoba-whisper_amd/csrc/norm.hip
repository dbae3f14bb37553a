// LayerNorm, conv-stem re-layout and decoder embedding (HBM-bound row kernels).
#include <algorithm>
#include "kw_common.h"

namespace {

// ---- LayerNorm: one wave per row, row held in registers (two-pass mean/var), 16-B loads. ----------
// TF/models/whisper/modeling_whisper.py:371,377,434,443,446,642,790 (nn.LayerNorm, eps 1e-5).
constexpr int LN_MAXV = 8;  // float4 per lane -> dim <= 64*4*8 = 2048

// With ``delta`` (bf16, optional) the residual add of the producing linear is fused in front:
// x += delta is written back (the f32 residual stream), then normalised (modeling_whisper.py:398,407).
template <typename TOut>
__global__ __launch_bounds__(256) void layernorm_kernel(float* __restrict__ x, int64_t rows, int dim,
                                                        const float* __restrict__ g, const float* __restrict__ bta,
                                                        float eps, TOut* __restrict__ y, const bf16_t* __restrict__ delta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar: one row per wave
  if (row >= rows) return;
  float4* xr = reinterpret_cast<float4*>(x + row * dim);
  const ushort4* dr = delta ? reinterpret_cast<const ushort4*>(delta + row * dim) : nullptr;
  const int nv = dim >> 2;
  float4 v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * 64 + lane;
    if (c < nv) {
      v[i] = xr[c];
      if (dr) {
        const ushort4 dd = dr[c];
        v[i].x += bf2f(dd.x);
        v[i].y += bf2f(dd.y);
        v[i].z += bf2f(dd.z);
        v[i].w += bf2f(dd.w);
        xr[c] = v[i];
      }
      s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    } else {
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const float mean = wave_sum(s) / (float)dim;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * 64 + lane;
    if (c < nv) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
      q += (a * a + b * b) + (cc * cc + d * d);
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)dim + eps);
  TOut* yr = y + row * dim;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(bta);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * 64 + lane;
    if (c < nv) {
      const float4 gg = g4[c], bb = b4[c];
      float o0 = (v[i].x - mean) * rstd * gg.x + bb.x;
      float o1 = (v[i].y - mean) * rstd * gg.y + bb.y;
      float o2 = (v[i].z - mean) * rstd * gg.z + bb.z;
      float o3 = (v[i].w - mean) * rstd * gg.w + bb.w;
      if constexpr (sizeof(TOut) == 4) {
        reinterpret_cast<float4*>(yr)[c] = make_float4(o0, o1, o2, o3);
      } else {
        ushort4 o;
        o.x = f2bf(o0); o.y = f2bf(o1); o.z = f2bf(o2); o.w = f2bf(o3);
        reinterpret_cast<ushort4*>(yr)[c] = o;
      }
    }
  }
}

// ---- The same over a bf16 residual stream (the encoder's bf16 path): 16-B accesses of 8 elements, the
// row held in registers.  x += delta is rounded to bf16 -- the reference's residual add in a bf16 model
// (modeling_whisper.py:398,407 under torch_dtype=bfloat16) -- and the LayerNorm reads the rounded sum.
constexpr int LNB_MAXV = 4;  // 8-element chunks per lane -> dim <= 64*8*4 = 2048

template <typename TOut>
__global__ __launch_bounds__(256) void layernorm_bf16res_kernel(bf16_t* __restrict__ x, int64_t rows, int dim,
                                                                const float* __restrict__ g,
                                                                const float* __restrict__ bta, float eps,
                                                                TOut* __restrict__ y, const bf16_t* __restrict__ delta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar: one row per wave
  if (row >= rows) return;
  uint4* xr = reinterpret_cast<uint4*>(x + row * dim);
  const uint4* dr = delta ? reinterpret_cast<const uint4*>(delta + row * dim) : nullptr;
  const int nv = dim >> 3;
  uint4 raw[LNB_MAXV], draw[LNB_MAXV];
#pragma unroll
  for (int i = 0; i < LNB_MAXV; ++i) {  // every load of the row in flight first
    const int c = i * 64 + lane;
    if (c < nv) {
      raw[i] = xr[c];
      if (dr) draw[i] = dr[c];
    }
  }
  float v[LNB_MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LNB_MAXV; ++i) {
    const int c = i * 64 + lane;
    if (c < nv) {
      const uint32_t w[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[i][2 * e] = __uint_as_float(w[e] << 16);
        v[i][2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
      }
      if (dr) {
        const uint32_t d[4] = {draw[i].x, draw[i].y, draw[i].z, draw[i].w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[i][2 * e] = bf2f(f2bf(v[i][2 * e] + __uint_as_float(d[e] << 16)));
          v[i][2 * e + 1] = bf2f(f2bf(v[i][2 * e + 1] + __uint_as_float(d[e] & 0xffff0000u)));
          o[e] = pack_bf16x2(v[i][2 * e], v[i][2 * e + 1]);
        }
        xr[c] = make_uint4(o[0], o[1], o[2], o[3]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)dim;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LNB_MAXV; ++i) {
    const int c = i * 64 + lane;
    if (c < nv) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = v[i][e] - mean;
        q = fmaf(a, a, q);
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)dim + eps);
  TOut* yr = y + row * dim;
#pragma unroll
  for (int i = 0; i < LNB_MAXV; ++i) {
    const int c = i * 64 + lane;
    if (c < nv) {
      const float4 g0 = reinterpret_cast<const float4*>(g)[2 * c], g1 = reinterpret_cast<const float4*>(g)[2 * c + 1];
      const float4 b0 = reinterpret_cast<const float4*>(bta)[2 * c], b1 = reinterpret_cast<const float4*>(bta)[2 * c + 1];
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * gg[e] + bb[e];
      if constexpr (sizeof(TOut) == 4) {
        reinterpret_cast<float4*>(yr)[2 * c] = make_float4(o[0], o[1], o[2], o[3]);
        reinterpret_cast<float4*>(yr)[2 * c + 1] = make_float4(o[4], o[5], o[6], o[7]);
      } else {
        reinterpret_cast<uint4*>(yr)[c] = make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]),
                                                     pack_bf16x2(o[4], o[5]), pack_bf16x2(o[6], o[7]));
      }
    }
  }
}

// ---- mel [B][C][T] f32 -> [B][T+2][c_pad] (zero time padding rows and zero channel padding) ----
template <typename TOut>
__global__ __launch_bounds__(256) void mel_tm_kernel(const float* __restrict__ mel, int C, int T, int c_pad,
                                                     TOut* __restrict__ out) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int t0 = blockIdx.x * 32;  // output time row block (padded coordinates)
  const int c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, tp = t0 + tx;  // read mel[b][c][tp-1]
    float v = 0.f;
    if (c < C && tp >= 1 && tp <= T) v = mel[((int64_t)b * C + c) * T + (tp - 1)];
    tile[i][tx] = v;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int tp = t0 + i, c = c0 + tx;
    if (tp < T + 2 && c < c_pad) TypeIO<TOut>::st(out + ((int64_t)b * (T + 2) + tp) * c_pad + c, tile[tx][i]);
  }
}

// ---- decoder embedding: h = tok_emb[id] + pos_emb[pos] (f32 residual stream) ----------------------
// bf16 tables, d % 8 == 0, 16-B aligned rows: each thread one 8-column piece (16-B loads of both tables, two 16-B f32
// stores and one 16-B bf16 store); the same per-element arithmetic as embed_kernel below (bitwise equal)
__global__ __launch_bounds__(256) void embed_bf16x8_kernel(const int64_t* __restrict__ ids, int64_t ids_stride, int q_len,
                                                           const int32_t* __restrict__ cur_len, const bf16_t* __restrict__ tok,
                                                           const bf16_t* __restrict__ pos, int d, float* __restrict__ h,
                                                           bf16_t* __restrict__ hb) {
  const int r = blockIdx.x;  // b*q_len + i
  const int b = r / q_len, i = r - b * q_len;
  const int p = *cur_len - q_len + i;
  const int64_t id = ids[(int64_t)b * ids_stride + p];
  for (int c = 8 * threadIdx.x; c < d; c += 8 * blockDim.x) {
    const u32x4 t4 = *reinterpret_cast<const u32x4*>(tok + id * d + c);
    const u32x4 p4 = *reinterpret_cast<const u32x4*>(pos + (int64_t)p * d + c);
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(t4[e] << 16) + __uint_as_float(p4[e] << 16);
      v[2 * e + 1] = __uint_as_float(t4[e] & 0xffff0000u) + __uint_as_float(p4[e] & 0xffff0000u);
    }
    float* hr = h + (int64_t)r * d + c;
    *reinterpret_cast<f32x4*>(hr) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(hr + 4) = f32x4{v[4], v[5], v[6], v[7]};
    if (hb)
      *reinterpret_cast<u32x4*>(hb + (int64_t)r * d + c) =
          u32x4{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
  }
}

template <typename TW>
__global__ __launch_bounds__(256) void embed_kernel(const int64_t* __restrict__ ids, int64_t ids_stride, int q_len,
                                                    const int32_t* __restrict__ cur_len, const TW* __restrict__ tok,
                                                    const TW* __restrict__ pos, int d, float* __restrict__ h,
                                                    bf16_t* __restrict__ hb) {
  const int r = blockIdx.x;  // b*q_len + i
  const int b = r / q_len, i = r - b * q_len;
  const int p = *cur_len - q_len + i;
  const int64_t id = ids[(int64_t)b * ids_stride + p];
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    const float v = TypeIO<TW>::ld(tok + id * d + c) + TypeIO<TW>::ld(pos + (int64_t)p * d + c);
    h[(int64_t)r * d + c] = v;
    if (hb) hb[(int64_t)r * d + c] = f2bf(v);
  }
}

}  // namespace

extern "C" int kw_layernorm(float* x, int64_t rows, int64_t dim, const float* gamma, const float* beta,
                            float eps, void* y, int y_dtype, const void* delta, kw_stream_t stream) {
  if (!x || !gamma || !beta || !y || rows < 0 || dim <= 0 || dim % 4 != 0 || dim > 64 * 4 * LN_MAXV)
    return kw_set_error_msg(KW_EINVAL, "kw_layernorm: invalid arguments (dim % 4 == 0, dim <= 2048)");
  if (rows == 0) return KW_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (y_dtype == KW_DT_F32)
    hipLaunchKernelGGL(layernorm_kernel<float>, grid, dim3(256), 0, s, x, rows, (int)dim, gamma, beta, eps, (float*)y,
                       (const bf16_t*)delta);
  else
    hipLaunchKernelGGL(layernorm_kernel<bf16_t>, grid, dim3(256), 0, s, x, rows, (int)dim, gamma, beta, eps, (bf16_t*)y,
                       (const bf16_t*)delta);
  KW_CHECK_LAUNCH();
  return KW_OK;
}

extern "C" int kw_layernorm_bf16res(void* x, int64_t rows, int64_t dim, const float* gamma, const float* beta,
                                    float eps, void* y, int y_dtype, const void* delta, kw_stream_t stream) {
  if (!x || !gamma || !beta || !y || rows < 0 || dim <= 0 || dim % 8 != 0 || dim > 64 * 8 * LNB_MAXV ||
      (uintptr_t)x % 16 != 0 || (uintptr_t)y % 16 != 0 || (delta && (uintptr_t)delta % 16 != 0))
    return kw_set_error_msg(KW_EINVAL, "kw_layernorm_bf16res: invalid arguments (dim % 8 == 0, dim <= 2048, 16-B aligned)");
  if (rows == 0) return KW_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (y_dtype == KW_DT_F32)
    hipLaunchKernelGGL(layernorm_bf16res_kernel<float>, grid, dim3(256), 0, s, (bf16_t*)x, rows, (int)dim, gamma, beta,
                       eps, (float*)y, (const bf16_t*)delta);
  else
    hipLaunchKernelGGL(layernorm_bf16res_kernel<bf16_t>, grid, dim3(256), 0, s, (bf16_t*)x, rows, (int)dim, gamma, beta,
                       eps, (bf16_t*)y, (const bf16_t*)delta);
  KW_CHECK_LAUNCH();
  return KW_OK;
}

extern "C" int kw_mel_to_time_major(const float* mel, int64_t B, int64_t C, int64_t T, int64_t c_pad, void* out,
                                    int out_dtype, kw_stream_t stream) {
  if (!mel || !out || B <= 0 || C <= 0 || T <= 0 || c_pad < C)
    return kw_set_error_msg(KW_EINVAL, "kw_mel_to_time_major: invalid arguments");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((T + 2 + 31) / 32), (unsigned)((c_pad + 31) / 32), (unsigned)B);
  if (out_dtype == KW_DT_F32)
    hipLaunchKernelGGL(mel_tm_kernel<float>, grid, dim3(256), 0, s, mel, (int)C, (int)T, (int)c_pad, (float*)out);
  else
    hipLaunchKernelGGL(mel_tm_kernel<bf16_t>, grid, dim3(256), 0, s, mel, (int)C, (int)T, (int)c_pad, (bf16_t*)out);
  KW_CHECK_LAUNCH();
  return KW_OK;
}

extern "C" int kw_embed(int dtype, const int64_t* ids, int64_t ids_stride, int64_t B, int64_t q_len,
                        const int32_t* cur_len, const void* tok_emb, const void* pos_emb, int64_t d, float* h,
                        void* hb, kw_stream_t stream) {
  if (!ids || !cur_len || !tok_emb || !pos_emb || !h || B <= 0 || q_len <= 0 || d <= 0)
    return kw_set_error_msg(KW_EINVAL, "kw_embed: invalid arguments");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)(B * q_len));
  const bool vec = dtype == KW_DT_BF16 && d % 8 == 0 && (uintptr_t)tok_emb % 16 == 0 && (uintptr_t)pos_emb % 16 == 0 &&
                   (uintptr_t)h % 16 == 0 && (uintptr_t)hb % 16 == 0;
  if (vec) {
    const int64_t pieces = d / 8;
    const unsigned threads = (unsigned)std::min<int64_t>(256, (pieces + 63) / 64 * 64);
    hipLaunchKernelGGL(embed_bf16x8_kernel, grid, dim3(threads), 0, s, ids, ids_stride, (int)q_len, cur_len,
                       (const bf16_t*)tok_emb, (const bf16_t*)pos_emb, (int)d, h, (bf16_t*)hb);
  } else if (dtype == KW_DT_F32)
    hipLaunchKernelGGL(embed_kernel<float>, grid, dim3(256), 0, s, ids, ids_stride, (int)q_len, cur_len,
                       (const float*)tok_emb, (const float*)pos_emb, (int)d, h, (bf16_t*)hb);
  else
    hipLaunchKernelGGL(embed_kernel<bf16_t>, grid, dim3(256), 0, s, ids, ids_stride, (int)q_len, cur_len,
                       (const bf16_t*)tok_emb, (const bf16_t*)pos_emb, (int)d, h, (bf16_t*)hb);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
