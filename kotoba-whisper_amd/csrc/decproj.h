// A decode linear's output block computed inside another kernel's launch and handed on in-launch: the
// LayerNorm-fused projection of dec_linear_kernel<5, 1, true, KW_EPI_STORE, bf16> (declin.hip) for one 16-column
// block over M <= 32 rows, on a 256-thread (4-wave) workgroup, published as 8-byte {bf16 x 2, tag} granules
// (MI355X_MICROARCH price list, handoff-1to1: one sc1 store per granule, sc1 polls, untorn).
//
// Bitwise dec_linear's values: its 8-wave geometry (nv = ceil(nkt / 5) waves of 5 k-tiles, wave v owning
// k-tiles [nkt v / nv, nkt (v + 1) / nv)) runs as VIRTUAL waves v = wave + 4 r (r = 0, 1) -- the same
// fragments and MFMA order per v -- and the partial tiles and LayerNorm row sums are reduced in v order
// through LDS, as the launch reduces its waves.  A fragments come straight from the activation rows (L2).
#pragma once
#include "kw_common.h"

// development hook (tools/lab/qkv_stamps.hip defines it to record s_memrealtime per workgroup phase); no-op here
#ifndef KW_PROJ_STAMP
#define KW_PROJ_STAMP(slot)
#endif

namespace {

constexpr int PROJ_KTM = 5;                      // k-tiles per virtual wave (dec_linear's choose() for K <= 1280)
constexpr int PROJ_NV = 8;                       // virtual waves: K <= 8 x 5 x 32 = 1280
constexpr int PROJ_SCRATCH = 16384 + 2048 + 256;  // LDS: partial tiles [8][2][64] f32x4, row sums [8][32][2], stats

struct ProjArgs {
  const bf16_t* x;  // [M][ldx] bf16 (the LayerNorm's input rows)
  int64_t ldx;
  int M, K, N;
  float ln_eps;
  const float* colsum;  // [N] column sums of the gamma-folded weight
  const bf16x8* W;      // packed [N/16][K/32][64] fragments (kw_pack_weight)
  const float* bias;    // [N] or null
  float scale;          // multiplies columns < scale_cols (the query's head_dim^-0.5)
  int scale_cols;
  int* fault;  // the workspace's fault-injection word (tests): nonzero -> workgroup 0 skips its publish once
};

__host__ __device__ __forceinline__ bool proj_shape_ok(int64_t M, int64_t K) {
  return M >= 1 && M <= 32 && K % 32 == 0 && K / 32 <= PROJ_NV * PROJ_KTM;
}

// Workgroup cg's 16 columns: every wave takes part (one __syncthreads inside); wave 0 publishes
// gran[m * (N / 2) + n / 2] for rows m < M, tag 1 in the high word.
// ONESHOT: both virtual waves' weight AND activation fragments in flight at once (one memory round trip; 60 more
// registers -- for kernels already at <= 3 workgroups per CU); otherwise the second virtual wave's activation
// fragments load after the first's MFMAs.
template <bool ONESHOT>
__device__ __forceinline__ void proj_publish_granules(const ProjArgs& a, int cg, char* scratch,
                                                      unsigned long long* gran) {
  f32x4(*red)[2][64] = reinterpret_cast<f32x4(*)[2][64]>(scratch);           // [8][2][64]
  float(*rpart)[32][2] = reinterpret_cast<float(*)[32][2]>(scratch + 16384);  // [8][32][2]
  float(*rstat)[2] = reinterpret_cast<float(*)[2]>(scratch + 16384 + 2048);   // [32][2]
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int M = a.M, nkt = a.K >> 5;
  const int nv = (nkt + PROJ_KTM - 1) / PROJ_KTM;
  KW_PROJ_STAMP(0);
  const bf16_t* x0 = a.x + (int64_t)min(lane & 15, M - 1) * a.ldx + (lane >> 4) * 8;
  const bf16_t* x1 = a.x + (int64_t)min(16 + (lane & 15), M - 1) * a.ldx + (lane >> 4) * 8;
  const int n_e = min(cg * 16 + (lane & 15), a.N - 1);
  const float ebias = a.bias ? a.bias[n_e] : 0.f;
  const float ecsum = a.colsum[n_e];
  // the fault-injection word, loaded by every workgroup (unconditionally: no phi on a loaded value) with the
  // epilogue constants; only workgroup 0 acts on it (kw_dec_*_status_offset in include/kwhisper.h)
  const int fault = __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  // both virtual waves' weights in flight at once (HBM: the long round trip)
  bf16x8 wv[2][PROJ_KTM];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int v = min(wave + 4 * r, nv - 1);
    const int kt0 = (nkt * v) / nv, kt1 = (nkt * (v + 1)) / nv;
    const int ktl = max(kt1 - 1, kt0);
    if (wave + 4 * r < nv) {
#pragma unroll
      for (int u = 0; u < PROJ_KTM; ++u)
        wv[r][u] = __builtin_nontemporal_load(a.W + ((int64_t)cg * nkt + min(kt0 + u, ktl)) * 64 + lane);
    }
  }
  bf16x8 av[2][2][PROJ_KTM];  // [round][row half][k-tile]
  auto load_a = [&](int r) {
    const int v = min(wave + 4 * r, nv - 1);
    const int kt0 = (nkt * v) / nv, kt1 = (nkt * (v + 1)) / nv;
    const int ktl = max(kt1 - 1, kt0);
#pragma unroll
    for (int u = 0; u < PROJ_KTM; ++u) {
      const int kt = min(kt0 + u, ktl);
      av[r][0][u] = *reinterpret_cast<const bf16x8*>(x0 + kt * 32);
      av[r][1][u] = *reinterpret_cast<const bf16x8*>(x1 + kt * 32);
    }
  };
  load_a(0);
  if (ONESHOT && wave + 4 < nv) load_a(1);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int v = wave + 4 * r;
    if (v >= nv) break;
    const int kt0 = (nkt * v) / nv, kt1 = (nkt * (v + 1)) / nv;
    const bf16x8* w = wv[r];
    if (!ONESHOT && r) load_a(1);
    const bf16x8* a0 = av[r][0];
    const bf16x8* a1 = av[r][1];
    f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0, s0 = c0, s1 = c0, q0 = c0, q1 = c0;
#pragma unroll
    for (int u = 0; u < PROJ_KTM; ++u)
      if (kt0 + u < kt1) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], w[u], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], w[u], c1, 0, 0, 0);
      }
#pragma unroll
    for (int u = 0; u < PROJ_KTM; ++u)
      if (kt0 + u < kt1) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], ones, s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], ones, s1, 0, 0, 0);
        q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], a0[u], q0, 0, 0, 0);
        q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], a1[u], q1, 0, 0, 0);
      }
    if ((lane & 15) == 0) {  // row sums: every column of x.1 holds them
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        rpart[v][4 * (lane >> 4) + i][0] = s0[i];
        rpart[v][16 + 4 * (lane >> 4) + i][0] = s1[i];
      }
    }
    const int di = (lane & 15) - 4 * (lane >> 4);  // row sums of squares: the diagonal of x.x^T
    if (di >= 0 && di < 4) {
      rpart[v][lane & 15][1] = q0[di];
      rpart[v][16 + (lane & 15)][1] = q1[di];
    }
    red[v][0][lane] = c0;
    red[v][1][lane] = c1;
  }
  KW_PROJ_STAMP(1);
  __syncthreads();
  // r06: the two row halves' reduction, LayerNorm statistics and publish on waves 0 and 1 at once (each sums its half's
  // partial tiles in virtual-wave order and forms its rows' statistics itself: bitwise wave 0 alone doing both, as
  // kw_dec_linear's spread epilogue)
  if (wave >= 2) return;
  const int hh = wave;
  f32x4 c = red[0][hh][lane];
  for (int v = 1; v < nv; ++v) c += red[v][hh][lane];
  if (lane < 16) {
    const int m = 16 * hh + lane;
    float sx = 0.f, sq = 0.f;
    for (int v = 0; v < nv; ++v) {
      sx += rpart[v][m][0];
      sq += rpart[v][m][1];
    }
    const float inv = 1.f / (float)a.K;
    const float mean = sx * inv;
    rstat[m][0] = mean;
    rstat[m][1] = rsqrtf(fmaxf(sq * inv - mean * mean, 0.f) + a.ln_eps);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int n = cg * 16 + (lane & 15);
  const bool drop = cg == 0 && fault != 0;  // test hook: this launch's consumers of columns [0, 16) time out
  if (drop && wave == 0 && lane == 0) __hip_atomic_store(a.fault, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = 16 * hh + 4 * (lane >> 4) + r;
    float v = c[r];
    v = rstat[m][1] * (v - rstat[m][0] * ecsum);
    v += ebias;
    if (n < a.scale_cols) v *= a.scale;
    const uint32_t mine = f2bf(v);
    const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0xB1, 0xF, 0xF, false);  // lane ^ 1
    if ((lane & 1) == 0 && m < M && n < a.N && !drop)
      __hip_atomic_store(gran + (int64_t)m * (a.N / 2) + (n >> 1), (1ull << 32) | (mine | (other << 16)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  KW_PROJ_STAMP(2);
}

}  // namespace
