// Decode-step skinny GEMM (M <= 32 rows per launch; kw_gemv chunks up to 128) over pre-packed
// weights, gfx950.
//
// One 8-wave workgroup per 16 output columns (optionally x K splits).  Weights are packed into 1-KB
// v_mfma_f32_16x16x32_bf16 B-fragments ([N/16][K/32][64][8]) so every weight load is one fully
// coalesced 16-B/lane wave access.  Each wave streams its K-range in blocks of UNR fragments with the
// next block's loads in flight while the current block's MFMAs run (register double buffer), and
// every operand of the epilogue (bias, residual) is prefetched at kernel start: the kernel costs about
// one memory round trip plus transfer time.  The (optional) K-split seam publishes 32x16 partial tiles
// with write-through (sc1) stores; an arrival counter elects the last split, which sums the partials in
// FIXED order (deterministic; no fences, no float atomics -- MI355X_MICROARCH "Valid forms" row 1).
//
// Fusions for the decoder layer (TF/models/whisper/modeling_whisper.py:434-503):
//   * LayerNorm prologue (LNA): A = (h - mean) * rstd for the workgroup's K-range, formed in LDS from
//     the f32 residual stream h and per-row (sum, sum-of-squares) partials left by h's producer; the
//     LayerNorm's gamma/beta are folded into W and the bias when the weights are loaded;
//   * statistics epilogue (RESID): after h += A.W^T + b, the finishing workgroup writes its 16
//     columns' (sum, sum-of-squares) per row -- the next LayerNorm's statistics.
#include <stdlib.h>

#include "gemm_common.h"

namespace {
using namespace kwg;

constexpr int WAVES = 8;
constexpr int NT = WAVES * 64;
constexpr int UNR = 4;
constexpr int KR_MAX = 1280;   // LNA: largest K-range per workgroup held normalised in LDS
constexpr int TILE = 32 * 16;  // partial tile (rows x columns) per workgroup = NT elements
constexpr int CNT_MAX = 4096;  // arrival counters live at the START of the workspace (fixed offset)
static_assert(TILE == NT, "one tile element per thread");

template <int EPI, typename TC, bool LNA>
__global__ __launch_bounds__(NT) void gemv_kernel(GemmP p, int ksplit) {
  __shared__ __attribute__((aligned(16))) bf16_t xs[LNA ? 32 : 1][LNA ? KR_MAX + 8 : 8];
  __shared__ float red[WAVES][2][64][4];
  __shared__ float mstat[32][2];
  __shared__ float tile[32][17];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = blockIdx.x, sp = blockIdx.y;
  const int nkt = p.K >> 5;
  const int M = p.M;
  const int kb0 = (nkt * sp) / ksplit, kb1 = (nkt * (sp + 1)) / ksplit;  // this workgroup's k-tiles
  const int kt0 = kb0 + ((kb1 - kb0) * wave) / WAVES, kt1 = kb0 + ((kb1 - kb0) * (wave + 1)) / WAVES;
  const int nblk = (kt1 - kt0 + UNR - 1) / UNR;
  const bf16x8* Wp = reinterpret_cast<const bf16x8*>(p.W) + (int64_t)cb * nkt * 64 + lane;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const int arow = lane & 15, akoff = 8 * (lane >> 4);
  const int mrow0 = min(arow, M - 1), mrow1 = min(16 + arow, M - 1);
  const int ktl = max(kt1 - 1, kt0);  // clamp target (a valid k-tile even for an empty range)

  bf16x8 wA[UNR], wB[UNR], aA[UNR][2], aB[UNR][2];
  auto load_blk = [&](int blk, bf16x8(&w)[UNR], bf16x8(&a)[UNR][2]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int kt = min(kt0 + blk * UNR + u, ktl);
      w[u] = __builtin_nontemporal_load(Wp + (int64_t)kt * 64);
      if constexpr (!LNA) {
        a[u][0] = *reinterpret_cast<const bf16x8*>(A + (int64_t)mrow0 * p.lda + kt * 32 + akoff);
        a[u][1] = *reinterpret_cast<const bf16x8*>(A + (int64_t)mrow1 * p.lda + kt * 32 + akoff);
      }
    }
  };
  // 1. first weight block in flight
  if (nblk > 0) load_blk(0, wA, aA);

  // 2. epilogue operands prefetched (thread <-> one element of the 32x16 tile)
  const int em = tid >> 4, enl = tid & 15, en = cb * 16 + enl;
  const bool evalid = em < M && en < p.N;
  const float e_bias = p.bias ? p.bias[min(en, p.N - 1)] : 0.f;
  float e_old = 0.f;
  if constexpr (EPI == KW_EPI_RESID) e_old = reinterpret_cast<const float*>(p.C)[(int64_t)min(em, M - 1) * p.ldc + min(en, p.N - 1)];

  // 3. LayerNorm prologue (statistics and h loads issued together)
  if constexpr (LNA) {
    const int k0 = kb0 * 32;
    const int nq = (kb1 - kb0) * 8;  // float4 per row in range (<= 320)
    constexpr int J = 32 * (KR_MAX / 4) / NT;  // 20 float4 per thread at most
    float4 x[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int e = min(tid + j * NT, M * nq - 1);
      const int r = e / nq, c = (e - r * nq) * 4;
      x[j] = *reinterpret_cast<const float4*>(p.ln_h + (int64_t)r * p.lda + k0 + c);
    }
    {  // 16 lanes per row reduce the producer's slots (32 rows x 16 = 512 threads)
      const int r = tid >> 4, j = tid & 15;
      float s = 0.f, s2 = 0.f;
      if (r < M) {
        const float* st = p.ln_stats + (int64_t)r * p.ln_slots * 2;
        for (int i = j; i < p.ln_slots; i += 16) {
          s += st[2 * i];
          s2 += st[2 * i + 1];
        }
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
      if (r < M && j == 0) {
        const float mean = s / (float)p.K;
        const float var = fmaxf(s2 / (float)p.K - mean * mean, 0.f);
        mstat[r][0] = mean;
        mstat[r][1] = rsqrtf(var + p.ln_eps);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int e = tid + j * NT;
      if (e < M * nq) {
        const int r = e / nq, c = (e - r * nq) * 4;
        const float mean = mstat[r][0], rstd = mstat[r][1];
        ushort4 o;
        o.x = f2bf((x[j].x - mean) * rstd);
        o.y = f2bf((x[j].y - mean) * rstd);
        o.z = f2bf((x[j].z - mean) * rstd);
        o.w = f2bf((x[j].w - mean) * rstd);
        *reinterpret_cast<ushort4*>(&xs[r][c]) = o;
      }
    }
    __syncthreads();
  }

  // 4. main loop: block b's MFMAs run while block b+1's loads are in flight
  f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  auto mma_blk = [&](int blk, const bf16x8(&w)[UNR], const bf16x8(&a)[UNR][2]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int kt = kt0 + blk * UNR + u;
      if (kt < kt1) {
        bf16x8 a0, a1;
        if constexpr (LNA) {
          const int kk = (kt - kb0) * 32 + akoff;
          a0 = *reinterpret_cast<const bf16x8*>(&xs[mrow0][kk]);
          a1 = *reinterpret_cast<const bf16x8*>(&xs[mrow1][kk]);
        } else {
          a0 = a[u][0];
          a1 = a[u][1];
        }
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, w[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, w[u], acc1, 0, 0, 0);
      }
    }
  };
  for (int blk = 0; blk < nblk; blk += 2) {
    if (blk + 1 < nblk) load_blk(blk + 1, wB, aB);
    mma_blk(blk, wA, aA);
    if (blk + 1 < nblk) {
      if (blk + 2 < nblk) load_blk(blk + 2, wA, aA);
      mma_blk(blk + 1, wB, aB);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[wave][0][lane][r] = acc0[r];
    red[wave][1][lane][r] = acc1[r];
  }
  __syncthreads();

  // 5. this workgroup's partial for element (em, enl); MFMA C layout lane = ((m%16)/4)*16 + col, reg = m%4
  float part;
  {
    const int rb = em >> 4, l = ((em & 15) >> 2) * 16 + enl, r = em & 3;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) v += red[w][rb][l][r];
    part = v;
  }
  // 6. K-split seam
  if (ksplit > 1) {
    int* cnt = reinterpret_cast<int*>(p.ws);
    float* slab = reinterpret_cast<float*>(p.ws) + CNT_MAX + ((int64_t)cb * ksplit + sp) * TILE;
    __hip_atomic_store(slab + tid, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(cnt + cb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == ksplit - 1;
      if (last) __hip_atomic_store(cnt + cb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    const float* s0 = reinterpret_cast<const float*>(p.ws) + CNT_MAX + (int64_t)cb * ksplit * TILE;
    float v = 0.f;
    for (int s = 0; s < ksplit; ++s) v += __hip_atomic_load(s0 + s * TILE + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    part = v;
  }

  // 7. epilogue
  float v = part + e_bias;
  if (evalid) {
    if constexpr (EPI == KW_EPI_RESID) {
      v += e_old;
      reinterpret_cast<float*>(p.C)[(int64_t)em * p.ldc + en] = v;
    } else {
      if (p.gelu) v = gelu_erf(v);
      if (en < p.scale_cols) v *= p.scale;
      TypeIO<TC>::st(reinterpret_cast<TC*>(p.C) + (int64_t)em * p.ldc + en, v);
    }
  }
  if (EPI == KW_EPI_RESID && p.stats_out != nullptr) {
    tile[em][enl] = evalid ? v : 0.f;
    __syncthreads();
    const int ncb = (p.N + 15) >> 4;
    if (tid < M) {
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float x = tile[tid][j];
        s += x;
        s2 += x * x;
      }
      p.stats_out[((int64_t)tid * ncb + cb) * 2] = s;
      p.stats_out[((int64_t)tid * ncb + cb) * 2 + 1] = s2;
    }
  }
}

__global__ void pack_kernel(const bf16_t* __restrict__ W, int N, int K, bf16_t* __restrict__ out) {
  const int nkt = K >> 5;
  const int64_t total = (int64_t)((N + 15) >> 4) * nkt * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const int64_t tile = i >> 6;
    const int kt = (int)(tile % nkt);
    const int cb = (int)(tile / nkt);
    const int n = cb * 16 + (lane & 15);
    const int k = kt * 32 + 8 * (lane >> 4);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n < N) v = *reinterpret_cast<const uint4*>(W + (int64_t)n * K + k);
    reinterpret_cast<uint4*>(out)[i] = v;
  }
}

// K splits: 1 by default (measured with tools/kbench.py: at decode sizes the split seam costs more
// than the parallelism it adds); KW_GEMV_KSPLIT (env) overrides, for experiments only.
int host_ksplit(int64_t N, int64_t K, bool lna) {
  const int nkt = (int)(K / 32);
  int ks = 1;
  (void)N;
  if (const char* e = getenv("KW_GEMV_KSPLIT")) {
    const int f = atoi(e);
    if (f > 0) ks = f;
  }
  const int need = lna ? (int)((K + KR_MAX - 1) / KR_MAX) : 1;
  if (ks < need) ks = need;
  if (ks > nkt) ks = nkt;
  return ks < 1 ? 1 : ks;
}

template <int EPI, typename TC, bool LNA>
hipError_t launch3(const GemmP& p, int ks, hipStream_t s) {
  dim3 grid((p.N + 15) / 16, ks);
  hipLaunchKernelGGL((gemv_kernel<EPI, TC, LNA>), grid, dim3(NT), 0, s, p, ks);
  return hipGetLastError();
}

template <typename TC>
hipError_t launch_gemv(const GemmP& p, int epi, int ks, hipStream_t s) {
  const bool lna = p.ln_h != nullptr;
  if (epi == KW_EPI_RESID)
    return lna ? launch3<KW_EPI_RESID, float, true>(p, ks, s) : launch3<KW_EPI_RESID, float, false>(p, ks, s);
  return lna ? launch3<KW_EPI_STORE, TC, true>(p, ks, s) : launch3<KW_EPI_STORE, TC, false>(p, ks, s);
}

}  // namespace

extern "C" size_t kw_gemv_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  (void)M;
  const int64_t ncb = (N + 15) / 16;
  const int a = host_ksplit(N, K, true), b = host_ksplit(N, K, false);
  const int ks = a > b ? a : b;
  return (size_t)(CNT_MAX + ncb * ks * TILE) * sizeof(float);
}

extern "C" int kw_gemv(const kw_gemm_args* a, kw_stream_t stream) {
  int rc = check_common(a);
  if (rc) return rc;
  if (a->dtype != KW_DT_BF16) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_gemv: bf16 only (use kw_gemm for f32)");
  if (a->M > 128 || a->K % 32 != 0 || a->lda % 8 != 0 || a->epilogue == KW_EPI_HEADSPLIT)
    return kw_set_error_msg(KW_EINVAL, "kw_gemv: needs M <= 128, K % 32 == 0, lda % 8 == 0, no head-split");
  const bool lna = a->ln_h != nullptr;
  if (lna && (!a->ln_stats || a->ln_slots <= 0 || a->lda % 4 != 0))
    return kw_set_error_msg(KW_EINVAL, "kw_gemv: fused LayerNorm needs ln_stats and ln_slots > 0");
  if (a->stats_out && a->epilogue != KW_EPI_RESID)
    return kw_set_error_msg(KW_EINVAL, "kw_gemv: stats_out needs the RESID epilogue");
  if (a->M == 0) return KW_OK;
  const int ks = host_ksplit(a->N, a->K, lna);
  if (lna && (a->K / 32 + ks - 1) / ks * 32 > KR_MAX)
    return kw_set_error_msg(KW_EINVAL, "kw_gemv: fused LayerNorm K-range exceeds the LDS image");
  if (ks > 1 && (a->N + 15) / 16 > CNT_MAX) return kw_set_error_msg(KW_EINVAL, "kw_gemv: split-K needs N <= 65536");
  if (ks > 1 && (!a->workspace || a->ws_bytes < kw_gemv_workspace_bytes(a->M, a->N, a->K)))
    return kw_set_error_msg(KW_EINVAL, "kw_gemv: split-K needs a zeroed workspace of kw_gemv_workspace_bytes()");
  hipStream_t s = (hipStream_t)stream;
  const int64_t ncb = (a->N + 15) / 16;
  for (int64_t m0 = 0; m0 < a->M; m0 += 32) {  // 32-row chunks (weights re-streamed per chunk)
    GemmP p = to_params(a);
    p.M = (int)(a->M - m0 < 32 ? a->M - m0 : 32);
    p.A = reinterpret_cast<const bf16_t*>(a->A) + m0 * a->lda;
    const size_t csz = a->c_dtype == KW_DT_F32 ? 4 : 2;
    p.C = reinterpret_cast<char*>(a->C) + m0 * a->ldc * csz;
    if (lna) {
      p.ln_h = a->ln_h + m0 * a->lda;
      p.ln_stats = a->ln_stats + m0 * a->ln_slots * 2;
    }
    if (a->stats_out) p.stats_out = a->stats_out + m0 * ncb * 2;
    hipError_t e = a->c_dtype == KW_DT_F32 ? launch_gemv<float>(p, a->epilogue, ks, s)
                                           : launch_gemv<bf16_t>(p, a->epilogue, ks, s);
    if (e != hipSuccess) return kw_set_error(e);
  }
  return KW_OK;
}

extern "C" size_t kw_packed_weight_bytes(int64_t N, int64_t K) { return (size_t)((N + 15) / 16) * (size_t)K * 16 * 2; }

extern "C" int kw_pack_weight(const void* W, int64_t N, int64_t K, void* packed, kw_stream_t stream) {
  if (!W || !packed || N <= 0 || K <= 0 || K % 32 != 0)
    return kw_set_error_msg(KW_EINVAL, "kw_pack_weight: needs K % 32 == 0");
  hipLaunchKernelGGL(pack_kernel, dim3(1024), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)W, (int)N, (int)K,
                     (bf16_t*)packed);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
