// GEMMs for the Whisper hot path on gfx950 (CDNA4).
//
//  * gemm_bf16_kernel: 128x128x64 block tile, 4 waves (2x2, 64x64 each = 2x2 v_mfma_f32_32x32x16_bf16),
//    A and W tiles staged global->LDS with global_load_lds_dwordx4 (no VGPR round trip) into a
//    2-stage ring; the LDS image is lane-linear with an XOR swizzle applied on the SOURCE address
//    (slot = chunk ^ ((row>>1)&7)) so every ds_read_b128 fragment read is bank-conflict free;
//    XCD-aware bijective blockIdx remap.  Encoder QKV/out-proj/FFN, conv stem (im2col-free: the
//    time-major padded layout makes each im2col row a contiguous slice) and cross-K/V projection.
//  * gemm_f32_kernel: exact-f32 path (v_mfma_f32_32x32x2_f32 = bitwise fmaf chain) used by the
//    fp32 parity mode.
//  * gemv_packed_kernel: decode-step skinny GEMM (M <= 128).  Weights pre-packed into 1-KB
//    16x32 fragments so each wave streams W with perfectly coalesced 16-B/lane loads; activations
//    come from L2; 4 waves split K and reduce through LDS.  HBM-bound (weights read once per step).
// Shared epilogues: bias, exact GELU, column scale (q * head_dim^-0.5, modeling_whisper.py:309),
// row-periodic add (encoder positions, :621-624), residual add into the f32 stream, head-split store.
#include "gemm_common.h"

namespace {
using namespace kwg;

// ------------------------------------------------------------------------------------------------
// bf16 128x128x64, glds staging
// ------------------------------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 32 KB
constexpr int GEMM_LDS = 2 * STAGE_BYTES;       // 64 KB

__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

template <int EPI, typename TC>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int tiles_n = p.N / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = wgid / tiles_n, tn = wgid - (wgid / tiles_n) * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* W = reinterpret_cast<const bf16_t*>(p.W);
  const bf16_t* a_src[4];
  const bf16_t* b_src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = wave * 4 + i;
    const int rr = 8 * g + (lane >> 3);
    const int c = (lane & 7) ^ ((rr >> 1) & 7);
    const int m = min(m0 + rr, p.M - 1);
    a_src[i] = A + row_off(m, p.a_rpb, p.a_bs, p.lda) + c * 8;
    b_src[i] = W + (int64_t)(n0 + rr) * p.K + c * 8;
  }

  auto stage = [&](int s, int k0) {
    char* base = smem + s * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int g = wave * 4 + i;
      glds16(a_src[i] + k0, base + g * 1024);
      glds16(b_src[i] + k0, base + BM * BK * 2 + g * 1024);
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = p.K / BK;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * BK);
    const char* As = smem + (kt & 1) * STAGE_BYTES;
    const char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks * 2 + (lane >> 5);
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 32 + (lane & 31);
        a[i] = *reinterpret_cast<const bf16x8*>(As + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wn * 64 + j * 32 + (lane & 31);
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + (lane & 31);
    const float bias_n = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < p.M) epi_one<EPI, TC>(p, m, n, acc[i][j][r], bias_n);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// f32 64x64x16 (exact fp32 via v_mfma_f32_32x32x2_f32)
// ------------------------------------------------------------------------------------------------
constexpr int FBM = 64, FBN = 64, FBK = 16;

template <int EPI, typename TC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmP p) {
  __shared__ float As[FBM][FBK + 1];
  __shared__ float Bs[FBN][FBK + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * FBM, n0 = blockIdx.x * FBN;
  const float* A = reinterpret_cast<const float*>(p.A);
  const float* W = reinterpret_cast<const float*>(p.W);
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const int am = m0 + lr, bn = n0 + lr;
  const float* a_row = am < p.M ? A + row_off(am, p.a_rpb, p.a_bs, p.lda) : nullptr;
  const float* b_row = bn < p.N ? W + (int64_t)bn * p.K : nullptr;
  const int wm = wave >> 1, wn = wave & 1;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int k0 = 0; k0 < p.K; k0 += FBK) {
    float4 av = a_row ? *reinterpret_cast<const float4*>(a_row + k0 + lk) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 bv = b_row ? *reinterpret_cast<const float4*>(b_row + k0 + lk) : make_float4(0.f, 0.f, 0.f, 0.f);
    As[lr][lk + 0] = av.x; As[lr][lk + 1] = av.y; As[lr][lk + 2] = av.z; As[lr][lk + 3] = av.w;
    Bs[lr][lk + 0] = bv.x; Bs[lr][lk + 1] = bv.y; Bs[lr][lk + 2] = bv.z; Bs[lr][lk + 3] = bv.w;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < FBK; kk += 2) {
      const float a = As[wm * 32 + (lane & 31)][kk + (lane >> 5)];
      const float b = Bs[wn * 32 + (lane & 31)][kk + (lane >> 5)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= p.N) return;
  const float bias_n = p.bias ? p.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m < p.M) epi_one<EPI, TC>(p, m, n, acc[r], bias_n);
  }
}

template <typename TC>
hipError_t launch_bf16(const GemmP& p, int epi, hipStream_t s) {
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  switch (epi) {
    case KW_EPI_STORE:
      hipLaunchKernelGGL((gemm_bf16_kernel<KW_EPI_STORE, TC>), dim3(nwg), dim3(256), GEMM_LDS, s, p); break;
    case KW_EPI_RESID:
      hipLaunchKernelGGL((gemm_bf16_kernel<KW_EPI_RESID, float>), dim3(nwg), dim3(256), GEMM_LDS, s, p); break;
    default:
      hipLaunchKernelGGL((gemm_bf16_kernel<KW_EPI_HEADSPLIT, TC>), dim3(nwg), dim3(256), GEMM_LDS, s, p); break;
  }
  return hipGetLastError();
}

template <typename TC>
hipError_t launch_f32(const GemmP& p, int epi, hipStream_t s) {
  dim3 grid((p.N + FBN - 1) / FBN, (p.M + FBM - 1) / FBM);
  switch (epi) {
    case KW_EPI_STORE: hipLaunchKernelGGL((gemm_f32_kernel<KW_EPI_STORE, TC>), grid, dim3(256), 0, s, p); break;
    case KW_EPI_RESID: hipLaunchKernelGGL((gemm_f32_kernel<KW_EPI_RESID, float>), grid, dim3(256), 0, s, p); break;
    default: hipLaunchKernelGGL((gemm_f32_kernel<KW_EPI_HEADSPLIT, TC>), grid, dim3(256), 0, s, p); break;
  }
  return hipGetLastError();
}

}  // namespace

extern "C" int kw_gemm(const kw_gemm_args* a, kw_stream_t stream) {
  int rc = check_common(a);
  if (rc) return rc;
  if (a->M == 0) return KW_OK;
  const GemmP p = to_params(a);
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (a->dtype == KW_DT_BF16) {
    if (a->N % BN != 0 || a->K % BK != 0 || a->lda % 8 != 0)
      return kw_set_error_msg(KW_EINVAL, "kw_gemm(bf16): needs N % 128 == 0, K % 64 == 0, lda % 8 == 0");
    e = a->c_dtype == KW_DT_F32 ? launch_bf16<float>(p, a->epilogue, s) : launch_bf16<bf16_t>(p, a->epilogue, s);
  } else if (a->dtype == KW_DT_F32) {
    if (a->K % FBK != 0 || a->lda % 4 != 0)
      return kw_set_error_msg(KW_EINVAL, "kw_gemm(f32): needs K % 16 == 0, lda % 4 == 0");
    e = a->c_dtype == KW_DT_F32 ? launch_f32<float>(p, a->epilogue, s) : launch_f32<bf16_t>(p, a->epilogue, s);
  } else {
    return kw_set_error_msg(KW_EUNSUPPORTED, "kw_gemm: unsupported dtype");
  }
  if (e != hipSuccess) return kw_set_error(e);
  return KW_OK;
}
