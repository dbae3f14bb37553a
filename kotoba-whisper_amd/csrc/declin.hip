// Decode-step linear layers (a4/a5) over pre-packed weights, gfx950.
//
// One decode step multiplies B <= 32 rows (one token per sequence) by every decoder weight matrix:
// q/k/v (modeling_whisper.py:469-480), out-proj, cross q / out-proj (:323-335), fc1 / fc2 (:499-503)
// and the tied LM head proj_out (:1080).  At this size a linear is a weight STREAM: 3.3-13 MB per
// matrix read once, ~2 k-tiles of MFMA work per 1 KB loaded.  The kernel is built for latency:
//
//  * weights pre-packed into 1-KB v_mfma_f32_16x16x32_bf16 B-fragments [N/16][K/32][64 lanes][8]
//    (padded to a multiple of 32 columns), so every weight load is one coalesced 16-B/lane wave
//    access; each wave issues ALL its weight and activation loads up front (KTM k-tiles x NCB column
//    blocks, non-temporal weights) -- the kernel costs about one memory round trip plus transfer;
//  * a workgroup owns NCB x 16 columns (NCB = 2 reuses each activation fragment twice); its waves
//    split K and reduce through LDS; for few-column matrices with long K (fc2: N 1280, K 5120) KS
//    workgroups split K with a deterministic seam (write-through partial slabs, an arrival counter,
//    the last arriver sums the KS slabs in fixed order -- MI355X_MICROARCH "Valid forms" row 1);
//  * fused LayerNorm: a LayerNorm consumer's workgroup holds its 32 rows of the bf16 residual mirror
//    x whole (its waves split K), so it computes each row's sum and sum of squares itself on the
//    matrix cores (X.1 and the diagonal of X.X^T, fixed-order fp32) and applies the LayerNorm
//    algebraically,
//    LN(x) W'^T = rstd * (x W'^T - mean * colsum(W')): the MFMAs take x as it is and the LayerNorm
//    costs one multiply-add per output; gamma/beta are folded into W and bias at load time
//    (W' = W diag(gamma), b' = b + W beta) and colsum(W') is precomputed per column;
//  * RESID epilogue: h(f32) += acc + bias, plus the bf16 mirror hb = h (the next LayerNorm's operand).
// Everything is bitwise deterministic: no float atomics, every reduction in a fixed order.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "kw_common.h"

// development hooks (tools/lab/declin_lab.hip records s_memrealtime stamps through them); no-ops here
#ifndef KW_DEC_STAMP
#define KW_DEC_STAMP_DECL
#define KW_DEC_STAMP(slot)
#define KW_DEC_STAMP_FLUSH
#endif

namespace {

__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

constexpr int CNT_MAX = 4096;  // seam arrival counters at the start of the workspace
constexpr int MAXW = 8;        // waves per workgroup
constexpr int KSMAX = 8;       // K splits per column group (host-checked)
constexpr int ZMAX = 8;        // 32-row chunks per K-split launch (workspace sized for them)

struct DecP {
  const bf16_t* x;
  int64_t ldx;
  int ln;
  float ln_eps;
  const float* ln_colsum;
  const bf16x8* W;
  const float* bias;
  void* C;
  int64_t ldc;
  int gelu;
  float scale;
  int scale_cols;
  float* h;
  bf16_t* hb;
  int64_t ldh;
  int M, N, K;
  float* slab;
  int* cnt;
  int xlds;  // stage the activation rows through LDS (single-round grids and split-K slices)
  int zrows; // rows per grid z-chunk: 32, or 16 for narrow grids (row split, launch())
  int vec_epi;  // outputs in whole 16-B pieces (N % 16 == 0, 16-B aligned rows): the epilogue stores 16-B pieces
};

// One wave's 16 x 16 output block: lane holds rows mb + 4 (lane / 16) + r (r < 4) of column nb + lane % 16 (the MFMA C
// layout).  vec (DecP::vec_epi): staged row-major in stg (the wave's own 16 x 20 floats of LDS) and stored as whole
// 16-B pieces -- f32 rows of 4 columns (one per lane), bf16 rows of 8 (lanes 0..31) -- otherwise element by element;
// rows >= M and columns >= N are not stored.  RESID: h (f32) and its bf16 mirror hb; STORE: C of TC.  r06: the
// element stores wrote 16 columns x 4 rows of 2-4-B pieces per instruction.
template <int EPI, typename TC>
__device__ __forceinline__ void store_block16(const DecP& p, float (*stg)[20], const float (&v4)[4], int mb, int M,
                                              int nb, int lane) {
  if (p.vec_epi) {
#pragma unroll
    for (int r = 0; r < 4; ++r) stg[4 * (lane >> 4) + r][lane & 15] = v4[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr bool F32 = EPI == KW_EPI_RESID || sizeof(TC) == 4, BF16 = EPI == KW_EPI_RESID || sizeof(TC) == 2;
    if constexpr (F32) {
      float* dst = EPI == KW_EPI_RESID ? p.h : reinterpret_cast<float*>(p.C);
      const int64_t ld = EPI == KW_EPI_RESID ? p.ldh : p.ldc;
      const int ml = lane >> 2, q = lane & 3, m = mb + ml;
      if (m < M && nb + 4 * q < p.N)
        *reinterpret_cast<f32x4*>(dst + (int64_t)m * ld + nb + 4 * q) = *reinterpret_cast<const f32x4*>(&stg[ml][4 * q]);
    }
    if constexpr (BF16) {
      bf16_t* dst = EPI == KW_EPI_RESID ? p.hb : reinterpret_cast<bf16_t*>(p.C);
      const int64_t ld = EPI == KW_EPI_RESID ? p.ldh : p.ldc;
      const int ml = lane >> 1, q = lane & 1, m = mb + ml;
      if (lane < 32 && m < M && nb + 8 * q < p.N) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&stg[ml][8 * q]);
        const f32x4 b = *reinterpret_cast<const f32x4*>(&stg[ml][8 * q + 4]);
        *reinterpret_cast<u32x4*>(dst + (int64_t)m * ld + nb + 8 * q) =
            u32x4{pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(b[0], b[1]), pack_bf16x2(b[2], b[3])};
      }
    }
  } else {
    const int n = nb + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mb + 4 * (lane >> 4) + r;
      if (n >= p.N || m >= M) continue;
      if constexpr (EPI == KW_EPI_RESID) {
        p.h[(int64_t)m * p.ldh + n] = v4[r];
        p.hb[(int64_t)m * p.ldh + n] = f2bf(v4[r]);
      } else {
        TypeIO<TC>::st(reinterpret_cast<TC*>(p.C) + (int64_t)m * p.ldc + n, v4[r]);
      }
    }
  }
}

// H2: the second 16-row half of the tile exists (false: a row-split chunk of <= 16 rows -- its a1 / c1 / LayerNorm
// statistics are never loaded or computed, which frees the registers for two workgroups per CU)
template <int KTM, int NCB, bool LNA, int EPI, typename TC, bool H2 = true>
__device__ __forceinline__ void dec_linear_body(DecP p, const int ksn, const int cg, const int ks, const int nw) {
  __shared__ f32x4 red[MAXW][NCB][2][64];
  __shared__ float rpart[MAXW][32][2];  // LayerNorm: per-wave row (sum, sum of squares)
  __shared__ float rstat[32][2];     // LayerNorm: (mean, rstd) per row
  extern __shared__ __attribute__((aligned(16))) char xs[];  // activation image (x_lds_bytes)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform (scalar branches)
  const int nkt = p.K >> 5;
  const int nsl = ksn * nw, sl = ks * nw + wave;
  const int kt0 = (nkt * sl) / nsl, kt1 = (nkt * (sl + 1)) / nsl;  // <= KTM k-tiles (host-checked)
  const int ktl = max(kt1 - 1, kt0);
  const int M = p.M;
  const int arow = lane & 15;
  KW_DEC_STAMP_DECL
  KW_DEC_STAMP(0);

  // 1. every load of this wave in flight: weights (non-temporal) into registers, and the workgroup's
  //    activation rows x[0:32][its k-range] into LDS by LDS-DMA in whole contiguous 1-KB pieces
  //    (the MFMA fragment pattern -- 16 rows x 64 B per load, every workgroup reading the same rows --
  //    is 2-3x slower to land from L2 than contiguous pieces).  LDS image: 32 rows of cpr 16-B chunks
  //    plus one pad chunk per row (odd row stride: the fragment reads are bank-conflict free).
  // (a row-split chunk, H2 = false: the other 16-row chunk's workgroup -- blockIdx 80 apart, the same XCD -- reads the
  // same weight slice, so it is loaded with the default policy and the second read can hit that XCD's L2; r04's nt
  // loads fetched 1.23x the o / xo weights from memory, profiles/r04p_pmc_fetch.csv)
  bf16x8 w[NCB][KTM], a0[KTM], a1[KTM];
#pragma unroll
  for (int c = 0; c < NCB; ++c)
#pragma unroll
    for (int u = 0; u < KTM; ++u) {
      const bf16x8* src = p.W + ((int64_t)(cg * NCB + c) * nkt + min(kt0 + u, ktl)) * 64 + lane;
      w[c][u] = H2 ? __builtin_nontemporal_load(src) : *src;
    }
  const int wkt0 = (nkt * ks) / ksn, wkt1 = (nkt * (ks + 1)) / ksn;  // this workgroup's k-tiles
  const int cpr = (wkt1 - wkt0) * 4, cprp = cpr + 1;
  const bool xlds = p.xlds;
  if (xlds) {
    // <= 16 rows: only the pieces of rows 0..15 (the second row half's fragments then hold stale LDS, and its
    // output rows -- all >= M -- are discarded; every row of an MFMA tile is independent of the others)
    const int ninst = ((M <= 16 ? 16 : 32) * cprp + 63) / 64;
    const float inv = 1.0f / (float)cprp;
    const bf16_t* xk = p.x + (int64_t)wkt0 * 32;
    for (int j = wave; j < ninst; j += nw) {
      const int pidx = j * 64 + lane;
      int row = (int)(((float)pidx + 0.5f) * inv);
      int cs = pidx - row * cprp;
      if (cs < 0) { --row; cs += cprp; }
      if (cs >= cprp) { ++row; cs -= cprp; }
      if (row > 31) { row = 31; cs = 0; }  // tail of the last piece: any valid source
      if (cs >= cpr) cs = cpr - 1;         // the pad chunk
      glds16(xk + (int64_t)min(row, M - 1) * p.ldx + cs * 8, xs + j * 1024);
    }
  }
  // epilogue operands of wave 0 (lane <-> column lane&15, rows 4*(lane>>4)+r and 16+...), loaded with
  // the operands so the epilogue never waits on a memory round trip: bias, LayerNorm column sums and
  // (RESID) the residual rows
  // r06: with the epilogue spread over the tile's J = NCB x row-half jobs (one wave each: step 4), every job wave
  // loads the residual rows too (16 floats per lane from L2; it keeps only its job's four)
  constexpr int HH = H2 ? 2 : 1, J = NCB * HH;
  const bool spread = J > 1 && ksn == 1 && nw >= J;
  float hold[NCB][2][4], ebias[NCB], ecsum[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int n = min((cg * NCB + c) * 16 + (lane & 15), p.N - 1);
    ebias[c] = p.bias ? p.bias[n] : 0.f;
    ecsum[c] = LNA ? p.ln_colsum[n] : 0.f;
  }
  if constexpr (EPI == KW_EPI_RESID) {
    if (spread ? wave < J : wave == 0) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const int n = min((cg * NCB + c) * 16 + (lane & 15), p.N - 1);
#pragma unroll
        for (int hh = 0; hh < (H2 ? 2 : 1); ++hh)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = min(16 * hh + 4 * (lane >> 4) + r, M - 1);
            hold[c][hh][r] = p.h[(int64_t)m * p.ldh + n];
          }
      }
    }
  }

  if (xlds) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int u = 0; u < KTM; ++u) {
      const int pos = (arow * cprp) + (min(kt0 + u, ktl) - wkt0) * 4 + (lane >> 4);
      a0[u] = *reinterpret_cast<const bf16x8*>(xs + pos * 16);
      if constexpr (H2) a1[u] = *reinterpret_cast<const bf16x8*>(xs + (pos + 16 * cprp) * 16);
    }
  } else {
    const int r0 = min(arow, M - 1), r1 = min(16 + arow, M - 1), akoff = 8 * (lane >> 4);
#pragma unroll
    for (int u = 0; u < KTM; ++u) {
      const int k = min(kt0 + u, ktl) * 32 + akoff;
      a0[u] = *reinterpret_cast<const bf16x8*>(p.x + (int64_t)r0 * p.ldx + k);
      if constexpr (H2) a1[u] = *reinterpret_cast<const bf16x8*>(p.x + (int64_t)r1 * p.ldx + k);
    }
  }

  // 2. MFMA over this wave's k-tiles (raw operand: the LayerNorm is applied in the epilogue)
  KW_DEC_STAMP(1);
  f32x4 c0[NCB], c1[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    c0[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    c1[c] = c0[c];
  }
#pragma unroll
  for (int u = 0; u < KTM; ++u) {
    if (kt0 + u < kt1) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        c0[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], w[c][u], c0[c], 0, 0, 0);
        if constexpr (H2) c1[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], w[c][u], c1[c], 0, 0, 0);
      }
    }
  }

  // 3. LayerNorm statistics of the 32 rows (the workgroup's waves cover K: host-checked, ksn == 1), on
  //    the matrix cores: X.1 gives the row sums, X.X^T's diagonal the row sums of squares (the A
  //    fragment of X is also the B fragment of X^T); fixed-order fp32 accumulation, waves summed in
  //    order through LDS
  if constexpr (LNA) {
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
    f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0, q0 = s0, q1 = s0;
#pragma unroll
    for (int u = 0; u < KTM; ++u)
      if (kt0 + u < kt1) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], ones, s0, 0, 0, 0);
        if constexpr (H2) s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], ones, s1, 0, 0, 0);
        q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], a0[u], q0, 0, 0, 0);
        if constexpr (H2) q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], a1[u], q1, 0, 0, 0);
      }
    // C layout: lane holds rows 4*(lane>>4)+i, column lane&15
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        rpart[wave][4 * (lane >> 4) + i][0] = s0[i];
        if constexpr (H2) rpart[wave][16 + 4 * (lane >> 4) + i][0] = s1[i];
      }
    }
    const int di = (lane & 15) - 4 * (lane >> 4);  // diagonal element of this lane, if any
    if (di >= 0 && di < 4) {
      rpart[wave][lane & 15][1] = q0[di];
      if constexpr (H2) rpart[wave][16 + (lane & 15)][1] = q1[di];
    }
  }

  // 4. reduce the waves' K slices (fixed order); wave 0 continues
  KW_DEC_STAMP(2);
  if (spread) {
    // r06: the tile's J (column block, row half) jobs -- fc1: 4 -- on waves 0..J-1 at once, each summing its 16 x 16
    // partial tiles in wave order, forming its row half's LayerNorm statistics itself and storing its piece (LDS is in
    // order within a wave; two jobs of one half write the same values): bitwise wave 0 alone, as the rows kernel's
    // spread epilogue (dec_linear_rows_kernel) -- fc1's reduction + epilogue 2.0 us on one wave (profiles/r06f_*)
    __shared__ __attribute__((aligned(16))) float stg[J][16][20];
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      red[wave][c][0][lane] = c0[c];
      if constexpr (H2) red[wave][c][1][lane] = c1[c];
    }
    __syncthreads();
    if (wave >= J) return;
    const int cj = wave / HH, hj = wave - cj * HH;
    if constexpr (LNA) {
      if (lane < 16) {
        const int m = 16 * hj + lane;
        float sx = 0.f, sq = 0.f;
        for (int w2 = 0; w2 < nw; ++w2) {
          sx += rpart[w2][m][0];
          sq += rpart[w2][m][1];
        }
        const float inv = 1.f / (float)p.K;
        const float mean = sx * inv;
        rstat[m][0] = mean;
        rstat[m][1] = rsqrtf(fmaxf(sq * inv - mean * mean, 0.f) + p.ln_eps);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    f32x4 acc = red[0][cj][hj][lane];
    for (int w2 = 1; w2 < nw; ++w2) acc += red[w2][cj][hj][lane];
    KW_DEC_STAMP(3);
    float bn = 0.f, cs = 0.f, hv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCB; ++c)
      if (c == cj) {
        bn = ebias[c];
        cs = ecsum[c];
#pragma unroll
        for (int hh = 0; hh < HH; ++hh)
          if (hh == hj)
#pragma unroll
            for (int r = 0; r < 4; ++r) hv[r] = hold[c][hh][r];
      }
    const int nb = (cg * NCB + cj) * 16;  // the job's first column
    const int n = nb + (lane & 15);
    float v4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * hj + 4 * (lane >> 4) + r;
      float v = acc[r];
      if constexpr (LNA) v = rstat[m][1] * (v - rstat[m][0] * cs);
      v += bn;
      if constexpr (EPI == KW_EPI_RESID) {
        v += hv[r];
      } else {
        if (p.gelu) v = sizeof(TC) == 2 ? gelu_bf16out(v) : gelu_erf(v);
        if (n < p.scale_cols) v *= p.scale;
      }
      v4[r] = v;
    }
    store_block16<EPI, TC>(p, stg[wave], v4, 16 * hj, M, nb, lane);
    KW_DEC_STAMP(4);
    KW_DEC_STAMP_FLUSH
    return;
  }
  if (nw > 1) {
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      red[wave][c][0][lane] = c0[c];
      if constexpr (H2) red[wave][c][1][lane] = c1[c];
    }
    __syncthreads();
    if (wave != 0) return;
    for (int w2 = 1; w2 < nw; ++w2)
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        c0[c] += red[w2][c][0][lane];
        if constexpr (H2) c1[c] += red[w2][c][1][lane];
      }
  }
  if constexpr (LNA) {  // wave 0: lane r < 32 sums row r's wave partials in wave order -> (mean, rstd)
    if (lane < 32) {
      float sx = 0.f, sq = 0.f;
      for (int w2 = 0; w2 < nw; ++w2) {
        sx += rpart[w2][lane][0];
        sq += rpart[w2][lane][1];
      }
      const float inv = 1.f / (float)p.K;
      const float mean = sx * inv;
      rstat[lane][0] = mean;
      rstat[lane][1] = rsqrtf(fmaxf(sq * inv - mean * mean, 0.f) + p.ln_eps);
    }
  }

  // 5. K-split seam: publish the partial tile write-through, count arrivals, the last one sums in order.  r06: each
  //    lane's two accumulator quads go out as two 16-B sc1 stores and come back as 16-B sc1 loads (the 4-B sc1 stores
  //    were one fabric write each, ~6x the 16-B form's time per byte: MI355X_MICROARCH "stores of each flavour"); the
  //    same values summed in the same order.  Slab: [column group][K split][NCB][row half][64 lanes][4] f32
  if (ksn > 1) {
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(p.slab + (int64_t)cg * ksn * (NCB * 512), (short)0,
                                                                         ksn * NCB * 512 * 4, 0x00020000);
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, c0[c]), srs, ((ks * NCB + c) * 128 + lane) * 16, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, c1[c]), srs, ((ks * NCB + c) * 128 + 64 + lane) * 16, 0, 16);
    }  // (aux 16 = sc1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) {
      const int prev = __hip_atomic_fetch_add(p.cnt + cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == ksn - 1;
      if (last) __hip_atomic_store(p.cnt + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = __shfl(last, 0, 64);
    if (!last) return;
    // every slab load in flight before the first add (fixed summation order q = 0, 1, ...); splits q >= ksn lie past
    // the buffer's range and load zeros, as the 4-B form's 0.f did
    f32x4 pv[KSMAX][NCB][2];
#pragma unroll
    for (int q = 0; q < KSMAX; ++q)
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        pv[q][c][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(srs, ((q * NCB + c) * 128 + lane) * 16, 0, 16));
        pv[q][c][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(srs, ((q * NCB + c) * 128 + 64 + lane) * 16, 0, 16));
      }
#pragma unroll
    for (int c = 0; c < NCB; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = pv[0][c][0][r], v1 = pv[0][c][1][r];
#pragma unroll
        for (int q = 1; q < KSMAX; ++q) {
          v0 += pv[q][c][0][r];
          v1 += pv[q][c][1][r];
        }
        c0[c][r] = v0;
        c1[c][r] = v1;
      }
  }

  KW_DEC_STAMP(3);
  // 6. epilogue: MFMA C layout -> element (row 4*(lane>>4)+r [+16], column lane&15); from here on wave 0 runs alone
  float vals[NCB][2][4];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int n = (cg * NCB + c) * 16 + (lane & 15);
    const float bn = ebias[c];
    const float cs = ecsum[c];
#pragma unroll
    for (int hh = 0; hh < (H2 ? 2 : 1); ++hh) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * hh + 4 * (lane >> 4) + r;
        float v = hh ? c1[c][r] : c0[c][r];
        if constexpr (LNA) v = rstat[m][1] * (v - rstat[m][0] * cs);  // LN(x) W'^T
        v += bn;
        if constexpr (EPI == KW_EPI_RESID) {
          v += hold[c][hh][r];
        } else {
          if (p.gelu) v = sizeof(TC) == 2 ? gelu_bf16out(v) : gelu_erf(v);
          if (n < p.scale_cols) v *= p.scale;
        }
        vals[c][hh][r] = v;
      }
    }
  }
  constexpr int R = H2 ? 32 : 16;  // rows of the tile
  if (p.vec_epi) {
    // r06: the tile staged row-major in the (now free) reduction buffer, then stored as whole 16-B pieces -- f32 rows
    // 4 columns, bf16 rows 8 -- instead of 2-4-B stores of 16 columns x 4 rows per instruction (the same values)
    constexpr int SW = NCB * 16 + 4;  // staging row stride (floats): the 4 rows of one write 16 banks apart
    float* stg = reinterpret_cast<float*>(&red[0][0][0][0]);
#pragma unroll
    for (int c = 0; c < NCB; ++c)
#pragma unroll
      for (int hh = 0; hh < (H2 ? 2 : 1); ++hh)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(16 * hh + 4 * (lane >> 4) + r) * SW + c * 16 + (lane & 15)] = vals[c][hh][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n0 = cg * NCB * 16;
    constexpr bool F32 = EPI == KW_EPI_RESID || sizeof(TC) == 4, BF16 = EPI == KW_EPI_RESID || sizeof(TC) == 2;
    if constexpr (F32) {
      float* dst = EPI == KW_EPI_RESID ? p.h : reinterpret_cast<float*>(p.C);
      const int64_t ld = EPI == KW_EPI_RESID ? p.ldh : p.ldc;
#pragma unroll
      for (int i = 0; i < (R * NCB * 4 + 63) / 64; ++i) {
        const int pc = lane + 64 * i, m = pc / (NCB * 4), q = pc - m * (NCB * 4);
        if (pc < R * NCB * 4 && m < M && n0 + 4 * q < p.N)
          *reinterpret_cast<f32x4*>(dst + (int64_t)m * ld + n0 + 4 * q) = *reinterpret_cast<const f32x4*>(stg + m * SW + 4 * q);
      }
    }
    if constexpr (BF16) {
      bf16_t* dst = EPI == KW_EPI_RESID ? p.hb : reinterpret_cast<bf16_t*>(p.C);
      const int64_t ld = EPI == KW_EPI_RESID ? p.ldh : p.ldc;
#pragma unroll
      for (int i = 0; i < (R * NCB * 2 + 63) / 64; ++i) {
        const int pc = lane + 64 * i, m = pc / (NCB * 2), q = pc - m * (NCB * 2);
        if (pc < R * NCB * 2 && m < M && n0 + 8 * q < p.N) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(stg + m * SW + 8 * q);
          const f32x4 b = *reinterpret_cast<const f32x4*>(stg + m * SW + 8 * q + 4);
          *reinterpret_cast<u32x4*>(dst + (int64_t)m * ld + n0 + 8 * q) =
              u32x4{pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(b[0], b[1]), pack_bf16x2(b[2], b[3])};
        }
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      const int n = (cg * NCB + c) * 16 + (lane & 15);
#pragma unroll
      for (int hh = 0; hh < (H2 ? 2 : 1); ++hh)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * hh + 4 * (lane >> 4) + r;
          if (n >= p.N || m >= M) continue;
          const float v = vals[c][hh][r];
          if constexpr (EPI == KW_EPI_RESID) {
            p.h[(int64_t)m * p.ldh + n] = v;
            p.hb[(int64_t)m * p.ldh + n] = f2bf(v);
          } else {
            TypeIO<TC>::st(reinterpret_cast<TC*>(p.C) + (int64_t)m * p.ldc + n, v);
          }
        }
    }
  }
  KW_DEC_STAMP(4);
  KW_DEC_STAMP_FLUSH
}

template <int KTM, int NCB, bool LNA, int EPI, typename TC, bool H2 = true>
__global__ __launch_bounds__(512) void dec_linear_kernel(DecP p0, int ksn) {
  // blockIdx.z = 32-row chunk: a launch covers M rows as independent 32-row tiles (their workgroups
  // run concurrently and the repeat weight reads of the later chunks hit the caches)
  DecP p = p0;
  if (ksn > 1) {  // K-split seam: each chunk has its own counters and partial slabs
    p.cnt += blockIdx.z * gridDim.x;
    p.slab += (int64_t)blockIdx.z * gridDim.x * ksn * (NCB * 512);
  }
  if (blockIdx.z) {
    const int m0 = p0.zrows * blockIdx.z;
    p.M = min(p0.zrows, p0.M - m0);
    p.x += m0 * p0.ldx;
    if (p.C) p.C = reinterpret_cast<char*>(p.C) + (int64_t)m0 * p0.ldc * (sizeof(TC));
    if (p.h) p.h += m0 * p0.ldh;
    if (p.hb) p.hb += m0 * p0.ldh;
  } else {
    p.M = min(p0.zrows, p0.M);
  }
  dec_linear_body<KTM, NCB, LNA, EPI, TC, H2>(p, ksn, blockIdx.x, blockIdx.y, blockDim.x >> 6);
}

// More than 32 rows without a K split (prefill positions, beam rows): each workgroup keeps its
// columns' weight fragments in registers and walks ``zper`` 32-row chunks.  (One z-slice per chunk
// re-streams the weights per chunk and runs as many rounds of workgroups as there are chunks, each a
// full load round trip: 50 us for fc1 at 320 rows.)  Per chunk the arithmetic is dec_linear_kernel's
// operation for operation -- the same fragments, MFMA order, wave-ordered reduction and epilogue --
// so results are bitwise those of the chunked launch.
template <int KTM, int NCB, bool LNA, int EPI, typename TC>
__global__ __launch_bounds__(512) void dec_linear_rows_kernel(DecP p, int zper) {
  __shared__ f32x4 red[MAXW][NCB][2][64];
  __shared__ __attribute__((aligned(16))) float stg[MAXW][16][20];  // store_block16's staging, one block per wave
  __shared__ float rpart[MAXW][32][2];
  __shared__ float rstat[32][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
  const int cg = blockIdx.x;
  const int nkt = p.K >> 5;
  const int kt0 = (nkt * wave) / nw, kt1 = (nkt * (wave + 1)) / nw;  // <= KTM (host-checked)
  const int ktl = max(kt1 - 1, kt0);
  const int arow = lane & 15, akoff = 8 * (lane >> 4);
  const int nz = (p.M + 31) / 32;
  const int z0 = blockIdx.z * zper, z1 = min(nz, z0 + zper);
  bf16x8 w[NCB][KTM];
#pragma unroll
  for (int c = 0; c < NCB; ++c)
#pragma unroll
    for (int u = 0; u < KTM; ++u)
      w[c][u] = __builtin_nontemporal_load(p.W + ((int64_t)(cg * NCB + c) * nkt + min(kt0 + u, ktl)) * 64 + lane);
  float ebias[NCB], ecsum[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int n = min((cg * NCB + c) * 16 + (lane & 15), p.N - 1);
    ebias[c] = p.bias ? p.bias[n] : 0.f;
    ecsum[c] = LNA ? p.ln_colsum[n] : 0.f;
  }
  for (int z = z0; z < z1; ++z) {
    const int m0 = 32 * z, M = min(32, p.M - m0);
    const bf16_t* x = p.x + (int64_t)m0 * p.ldx;
    bf16x8 a0[KTM], a1[KTM];
    {
      const int r0 = min(arow, M - 1), r1 = min(16 + arow, M - 1);
#pragma unroll
      for (int u = 0; u < KTM; ++u) {
        const int k = min(kt0 + u, ktl) * 32 + akoff;
        a0[u] = *reinterpret_cast<const bf16x8*>(x + (int64_t)r0 * p.ldx + k);
        a1[u] = *reinterpret_cast<const bf16x8*>(x + (int64_t)r1 * p.ldx + k);
      }
    }
    // the residual values, loaded by the wave that writes them in the epilogue (NCB == 2: its job (c, hh))
    float hold[NCB][2][4];
    if constexpr (EPI == KW_EPI_RESID && NCB == 2) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const int n = min((cg * NCB + c) * 16 + (lane & 15), p.N - 1);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          if ((2 * c + hh) % nw == wave) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int m = min(16 * hh + 4 * (lane >> 4) + r, M - 1);
              hold[c][hh][r] = p.h[(int64_t)(m0 + m) * p.ldh + n];
            }
          }
      }
    } else if constexpr (EPI == KW_EPI_RESID) {
      if (wave == 0) {
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          const int n = min((cg * NCB + c) * 16 + (lane & 15), p.N - 1);
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int m = min(16 * hh + 4 * (lane >> 4) + r, M - 1);
              hold[c][hh][r] = p.h[(int64_t)(m0 + m) * p.ldh + n];
            }
        }
      }
    }
    f32x4 c0[NCB], c1[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      c0[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      c1[c] = c0[c];
    }
#pragma unroll
    for (int u = 0; u < KTM; ++u) {
      if (kt0 + u < kt1) {
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          c0[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], w[c][u], c0[c], 0, 0, 0);
          c1[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], w[c][u], c1[c], 0, 0, 0);
        }
      }
    }
    if constexpr (LNA) {  // row statistics on the matrix cores, as dec_linear_kernel step 3
      bf16x8 ones;
#pragma unroll
      for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
      f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0, q0 = s0, q1 = s0;
#pragma unroll
      for (int u = 0; u < KTM; ++u)
        if (kt0 + u < kt1) {
          s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], ones, s0, 0, 0, 0);
          s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], ones, s1, 0, 0, 0);
          q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], a0[u], q0, 0, 0, 0);
          q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], a1[u], q1, 0, 0, 0);
        }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          rpart[wave][4 * (lane >> 4) + i][0] = s0[i];
          rpart[wave][16 + 4 * (lane >> 4) + i][0] = s1[i];
        }
      }
      const int di = (lane & 15) - 4 * (lane >> 4);
      if (di >= 0 && di < 4) {
        rpart[wave][lane & 15][1] = q0[di];
        rpart[wave][16 + (lane & 15)][1] = q1[di];
      }
    }
    if (NCB == 2 || nw > 1) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        red[wave][c][0][lane] = c0[c];
        red[wave][c][1][lane] = c1[c];
      }
    }
    __syncthreads();
    if constexpr (NCB == 2) {
      // two column blocks: the epilogue's four jobs -- (column block c, row half hh) -- spread over the waves (job
      // = wave + i nw), each summing its partial tiles over the waves in wave order as wave 0 alone does below and
      // forming its row half's LayerNorm statistics itself (LDS is in order within a wave; two jobs of one half
      // write the same values): bitwise the same results.  fc1 at 320 rows 41.4 -> 36.5 us; one column block keeps
      // wave 0 alone, which measured faster there (profiles/r05al_rows_epilogue_ab.txt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int job = wave + i * nw;
        if (job >= 4) break;
        const int c = job >> 1, hh = job & 1;
        if constexpr (LNA) {
          if (lane < 16) {
            const int m = 16 * hh + lane;
            float sx = 0.f, sq = 0.f;
            for (int w2 = 0; w2 < nw; ++w2) {
              sx += rpart[w2][m][0];
              sq += rpart[w2][m][1];
            }
            const float inv = 1.f / (float)p.K;
            const float mean = sx * inv;
            rstat[m][0] = mean;
            rstat[m][1] = rsqrtf(fmaxf(sq * inv - mean * mean, 0.f) + p.ln_eps);
          }
        }
        f32x4 acc = red[0][c][hh][lane];
        for (int w2 = 1; w2 < nw; ++w2) acc += red[w2][c][hh][lane];
        const int n = (cg * NCB + c) * 16 + (lane & 15);
        const float bn = ebias[c];
        const float cs = ecsum[c];
        float v4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * hh + 4 * (lane >> 4) + r;
          float v = acc[r];
          if constexpr (LNA) v = rstat[m][1] * (v - rstat[m][0] * cs);
          v += bn;
          if constexpr (EPI == KW_EPI_RESID) {
            v += hold[c][hh][r];
          } else {
            if (p.gelu) v = sizeof(TC) == 2 ? gelu_bf16out(v) : gelu_erf(v);
            if (n < p.scale_cols) v *= p.scale;
          }
          v4[r] = v;
        }
        store_block16<EPI, TC>(p, stg[wave], v4, m0 + 16 * hh, m0 + M, (cg * NCB + c) * 16, lane);
      }
    } else if (wave == 0) {
      for (int w2 = 1; w2 < nw; ++w2)
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          c0[c] += red[w2][c][0][lane];
          c1[c] += red[w2][c][1][lane];
        }
      if constexpr (LNA) {
        if (lane < 32) {
          float sx = 0.f, sq = 0.f;
          for (int w2 = 0; w2 < nw; ++w2) {
            sx += rpart[w2][lane][0];
            sq += rpart[w2][lane][1];
          }
          const float inv = 1.f / (float)p.K;
          const float mean = sx * inv;
          rstat[lane][0] = mean;
          rstat[lane][1] = rsqrtf(fmaxf(sq * inv - mean * mean, 0.f) + p.ln_eps);
        }
      }
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const int n = (cg * NCB + c) * 16 + (lane & 15);
        const float bn = ebias[c];
        const float cs = ecsum[c];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float v4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = 16 * hh + 4 * (lane >> 4) + r;
            float v = hh ? c1[c][r] : c0[c][r];
            if constexpr (LNA) v = rstat[m][1] * (v - rstat[m][0] * cs);
            v += bn;
            if constexpr (EPI == KW_EPI_RESID) {
              v += hold[c][hh][r];
            } else {
              if (p.gelu) v = sizeof(TC) == 2 ? gelu_bf16out(v) : gelu_erf(v);
              if (n < p.scale_cols) v *= p.scale;
            }
            v4[r] = v;
          }
          store_block16<EPI, TC>(p, stg[0], v4, m0 + 16 * hh, m0 + M, (cg * NCB + c) * 16, lane);
        }
      }
    }
    __syncthreads();  // red / rpart / rstat / stg are rewritten by the next chunk
  }
}

// LM head over 33..LMR_MAXROWS rows (beam rows: 64 items x 5 beams = 320) as a GEMM: workgroup = 64
// columns (one 16-column block per wave, all of K) x ALL rows.  Per k-tile the workgroup stages the
// rows' 32-wide activation slice in LDS once (LDS-DMA, double-buffered, XOR-swizzled for conflict-free
// fragment reads) and every wave multiplies it by its one weight fragment (1 KB, streamed once from HBM,
// the next k-tile's in flight): no cross-wave reduction, no weight re-read per row chunk (the rows
// kernel re-reads the activations per 32 columns and reduces per chunk: 258 us at 320 rows).  The
// LayerNorm statistics accumulate from the same LDS slices (f32, k order); epilogue as the folded
// LayerNorm of dec_linear_kernel.  Results agree with the 32-row kernels to f32 summation order.
constexpr int LMR_MAXROWS = 320, LMR_NZ = LMR_MAXROWS / 32;

__device__ __forceinline__ bf16x8 lmr_lds_read(const char* p) {
  // inline asm: a builtin LDS read after an LDS-DMA would get an s_waitcnt vmcnt(0) (the compiler
  // cannot tell the slice being read from the ones in flight); lmr waits are explicit lgkmcnt counts
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p)
               : "memory");
  return v;
}
__device__ __forceinline__ void lmr_barrier() {  // raw s_barrier: no implicit vmcnt(0) drain
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// NWV waves (16 columns each); G 16-B LDS-DMA pieces per lane per slice (a slice holds 16 NWV G rows); NZ 32-row
// chunks computed.  NWV = 4: three slices (two staged ahead), two workgroups per CU; NWV = 8: five slices (four
// staged ahead), one workgroup per CU -- the same eight waves per CU, each slice staged once per CU instead of twice.
template <int NWV, int G, int NZ>
__global__ __launch_bounds__(64 * NWV) void lm_head_rows_kernel(DecP p) {
  constexpr int NBUF = NWV == 8 ? 5 : 3, LEAD = NBUF - 1, PD = 8;  // slices in LDS, weight fragments in flight
  constexpr int SLICE = 1024 * NWV * G;                            // bytes per slice (64 B per row)
  static_assert(NZ <= LMR_NZ && 32 * NZ <= 16 * NWV * G && PD > LEAD, "lm_head_rows_kernel geometry");
  __shared__ __attribute__((aligned(16))) char abuf[NBUF][SLICE];
  __shared__ float rsum[LMR_MAXROWS], rsq[LMR_MAXROWS];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform (scalar branches)
  const int M = p.M, nkt = p.K >> 5, nz = (M + 31) / 32;
  const int n_cb = (p.N + 15) / 16;
  const int cb = min(blockIdx.x * NWV + wave, n_cb - 1);
  // staging: piece j (16 B) = row j >> 2, LDS chunk j & 3, holding source chunk (j & 3) ^ ((row >> 2) & 3)
  auto stage = [&](int buf, int kt) {
    char* dst = abuf[buf];
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int j0 = wave * 64 + 64 * NWV * i;
      const int j = j0 + lane, row = j >> 2, ch = (j & 3) ^ ((row >> 2) & 3);
      glds16(p.x + (int64_t)min(row, M - 1) * p.ldx + kt * 32 + ch * 8, dst + j0 * 16);
    }
  };
  f32x4 acc0[LMR_NZ], acc1[LMR_NZ];
#pragma unroll
  for (int z = 0; z < LMR_NZ; ++z) {
    acc0[z] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc1[z] = acc0[z];
  }
  // row statistics from the fragments: wave w sums chunks z = w, w + NWV, ... (slot z / NWV); lane
  // (fr, fc) holds 8 values of rows 32z + fr and 32z + 16 + fr
  constexpr int NSL = (LMR_NZ + NWV - 1) / NWV;
  float ss[NSL][2], sq[NSL][2];
#pragma unroll
  for (int t = 0; t < NSL; ++t) ss[t][0] = ss[t][1] = sq[t][0] = sq[t][1] = 0.f;
  const bf16x8* W = p.W + (int64_t)cb * nkt * 64 + lane;
  // (rows past M are clamped copies, never stored)
  const int fr = lane & 15, fc = lane >> 4;  // fragment row within a 16-row block, 16-B chunk
  // Branch-free k loop (the compiler's own vmcnt bookkeeping then stays exact): the slice and weight
  // prefetches are clamped to the last k-tile instead of skipped.  Issue order: W(0 .. PD-LEAD-1), then
  // S(i), W(PD-LEAD+i) for i < LEAD | k-tile kt: S(kt+LEAD), W(kt+PD); so at the top of k-tile kt exactly
  // LEAD - 1 slices (G pieces each) and LEAD weight fragments are younger than S(kt), and W(kt) is older.
  // nkt % PD == 0 (host-checked).  (NWV = 4: W(0..5), S(0), W(6), S(1), W(7); vmcnt(G + 2).)
  constexpr int YOUNGER = G * (LEAD - 1) + LEAD;
  bf16x8 wr[PD];
#pragma unroll
  for (int u = 0; u < PD - LEAD; ++u) wr[u] = __builtin_nontemporal_load(W + (int64_t)min(u, nkt - 1) * 64);
#pragma unroll
  for (int i = 0; i < LEAD; ++i) {
    stage(i, min(i, nkt - 1));
    wr[PD - LEAD + i] = __builtin_nontemporal_load(W + (int64_t)min(PD - LEAD + i, nkt - 1) * 64);
  }
  for (int kb = 0; kb < nkt; kb += PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int kt = kb + u;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(YOUNGER) : "memory");
      lmr_barrier();
      stage((kt + LEAD) % NBUF, min(kt + LEAD, nkt - 1));
      const char* a = abuf[kt % NBUF];
      bf16x8 fa[2][2];
      auto rd = [&](int z, bf16x8 (&f)[2]) {
        const int r0 = 32 * z + fr, r1 = r0 + 16;
        f[0] = lmr_lds_read(a + r0 * 64 + ((fc ^ ((r0 >> 2) & 3)) << 4));
        f[1] = lmr_lds_read(a + r1 * 64 + ((fc ^ ((r1 >> 2) & 3)) << 4));
      };
      rd(0, fa[0]);
#pragma unroll
      for (int z = 0; z < NZ; ++z) {
        bf16x8(&f)[2] = fa[z & 1];
        if (z + 1 < NZ) {
          rd(z + 1, fa[(z + 1) & 1]);
          asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(f[0]), "+v"(f[1]));
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]));
        }
        acc0[z] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], wr[u], acc0[z], 0, 0, 0);
        acc1[z] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[1], wr[u], acc1[z], 0, 0, 0);
        if (z % NWV == wave) {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = (float)f[hh][e];
              ss[z / NWV][hh] += x;
              sq[z / NWV][hh] = fmaf(x, x, sq[z / NWV][hh]);
            }
        }
      }
      wr[u] = __builtin_nontemporal_load(W + (int64_t)min(kt + PD, nkt - 1) * 64);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the clamped tail prefetches)
  // finish the statistics: the 4 lanes of a row (fc = 0..3) in chunk order
#pragma unroll
  for (int t = 0; t < NSL; ++t) {
    const int z = wave + NWV * t;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      float a = ss[t][hh], b = sq[t][hh];
      const float a1 = __shfl_xor(a, 16, 64), b1 = __shfl_xor(b, 16, 64);
      const float a2 = __shfl_xor(a, 32, 64), b2 = __shfl_xor(b, 32, 64);
      const float a3 = __shfl_xor(a, 48, 64), b3 = __shfl_xor(b, 48, 64);
      if (fc == 0 && z < nz) {
        const int row = 32 * z + 16 * hh + fr;
        rsum[row] = (a + a1) + (a2 + a3);
        rsq[row] = (b + b1) + (b2 + b3);
      }
    }
  }
  __syncthreads();
  const int n = cb * 16 + fr;
  if (blockIdx.x * NWV + wave >= n_cb || n >= p.N) return;
  const float cs = p.ln_colsum[n], bn = p.bias ? p.bias[n] : 0.f;
  const float inv = 1.f / (float)p.K;
#pragma unroll
  for (int z = 0; z < LMR_NZ; ++z) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 32 * z + 16 * hh + 4 * fc + r;
        if (z < nz && m < M) {
          const float mean = rsum[m] * inv;
          const float rstd = rsqrtf(fmaxf(rsq[m] * inv - mean * mean, 0.f) + p.ln_eps);
          const float v = hh ? acc1[z][r] : acc0[z][r];
          reinterpret_cast<float*>(p.C)[(int64_t)m * p.ldc + n] = rstd * (v - mean * cs) + bn;
        }
      }
  }
}

// LM head (proj_out with the final LayerNorm folded, modeling_whisper.py:790,1080) as a persistent
// weight stream: the generic kernel above re-reads the 32 activation rows from L2 in every one of its
// 1,621 workgroups (as many L2 bytes as weight bytes) and runs 1.6 rounds of them.  Here each of
// ~256 workgroups loads its waves' activation fragments and the rows' LayerNorm statistics ONCE, then
// walks a contiguous run of column groups (2 x 16 columns each) with the NEXT TWO groups' weights in
// flight while the current one is reduced across waves and written (fixed-order sums: deterministic).
// r05: the epilogue's column sums / biases of the whole run are staged in LDS at the start (no
// epilogue load in the loop), each prefetch is pinned where it is written (sched_barrier: the scheduler had sunk
// the next group's loads below the current group's waits), and the per-group barrier is a raw s_barrier after an
// LDS-only wait (__syncthreads drained every load in flight, the prefetch included).
constexpr int LMH_KTM = 5;   // k-tiles per wave
constexpr int LMH_NCB = 2;   // column blocks per group
constexpr int LMH_MAXG = 8;  // column groups per workgroup (epilogue constants and the logits staged in LDS; host-checked)
constexpr int LMH_ECJ = 4;   // epilogue-constant columns staged per thread (host-checked: 64 * waves * 4 >= 32 * groups)
constexpr int LMH_MAX_ROWS = 32;  // rows up to which the LM head takes lm_head_kernel (weight groups: three in
                                  // registers, two in flight beside the one being multiplied)

__device__ __forceinline__ void lmh_barrier() {  // LDS writes visible, then s_barrier: global loads stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The greedy step fused into the LM head (AM = true, kw_dec_lm_greedy; TF generation/utils.py:2894-2937 without
// timestamps): each workgroup, after its run's logits are staged in LDS, takes every row's processed arg-max over the
// run's columns (SuppressTokens, SuppressTokensAtBegin when L == begin_index; first index on ties) and publishes it as
// one 8-byte {value, index} partial (sc1 store); the last workgroup to arrive (one agent-scope counter, MI355X_MICROARCH
// "Valid forms" row 1) merges each row's partials -- the comparison (value, then lower index) is a total order, so the
// token is the one kw_greedy_step's slice-ordered merge picks, NaN never winning -- and finishes the step exactly as
// greedy_step_split_kernel does (finished -> pad, ids[L], unfinished, n_unfinished, cur_len).  The logits store is
// optional (C may be null).
struct LmGreedy {
  const uint8_t* mask;     // [V] SuppressTokens
  const int32_t* bsup;     // SuppressTokensAtBegin ids
  int nbsup;
  int64_t* ids;
  int64_t ids_stride;
  int32_t* cur_len;
  int max_length, begin_index, eos_id, pad_id;
  int32_t* unfinished;
  int32_t* n_unfinished;
  unsigned long long* part;  // [M][gridDim.x] {f32 value bits, int32 index}
  int* arrive;               // arrival counter (zero before first use; re-armed by the last arriver)
  int* fin;                  // [M] row r's finished flag, published by workgroup r
};

// (value, index) order of the arg-max: greater value, then lower index; NaN never wins (kw_greedy_step's compares)
__device__ __forceinline__ void am_take(float& best, int& bi, float s, int v) {
  if (s > best || (s == best && v < bi)) {
    best = s;
    bi = v;
  }
}
__device__ __forceinline__ unsigned long long am_pack(float best, int bi) {
  return (unsigned long long)__float_as_uint(best) | ((unsigned long long)(unsigned)bi << 32);
}

// AM epilogue: the run's partial arg-max per row, the arrival count, and in the last workgroup the merge and the step
// bookkeeping.  Row r of a 16-lane group: lanes j = 0..15 take the run's columns j, j + 16, ...
template <int OBW>
__device__ __forceinline__ void lm_greedy_tail(const LmGreedy& sg, const float (*obuf)[OBW], const uint8_t* smask,
                                               int ncol, int n0, int M, int L, int row_fin) {
  const int tid = threadIdx.x, j = tid & 15, nth = blockDim.x;
  const bool first = L == sg.begin_index;
  const int G = gridDim.x;
  for (int r = tid >> 4; r < M; r += nth >> 4) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int col = j; col < ncol; col += 16) {
      const int n = n0 + col;
      float s = smask[col] ? -INFINITY : obuf[r][col];
      if (first)
        for (int i = 0; i < sg.nbsup; ++i)
          if (sg.bsup[i] == n) s = -INFINITY;
      am_take(best, bi, s, n);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      am_take(best, bi, ob, oi);
    }
    if (j == 0)
      __hip_atomic_store(sg.part + (int64_t)r * G + blockIdx.x, am_pack(best, bi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0 && (int)blockIdx.x < M) __hip_atomic_store(sg.fin + blockIdx.x, row_fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's partials drained before the barrier
  __shared__ int am_last, am_nunf;
  __syncthreads();
  if (tid == 0) {
    am_nunf = 0;
    am_last = __hip_atomic_fetch_add(sg.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
  }
  __syncthreads();
  if (!am_last) return;
  // the last arriver: row r's G partials over its 16 lanes and its finished flag (sc1 loads, all in flight before
  // the compares), then the step's bookkeeping
  int n_unf = 0;
  for (int r = tid >> 4; r < M; r += nth >> 4) {
    constexpr int PQ = 16;  // partials per lane: G <= 256 (host-checked)
    unsigned long long pv[PQ];
#pragma unroll
    for (int q = 0; q < PQ; ++q)
      pv[q] = __hip_atomic_load(sg.part + (int64_t)r * G + min(j + 16 * q, G - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int fin = __hip_atomic_load(sg.fin + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < PQ; ++q)
      if (j + 16 * q < G) am_take(best, bi, __uint_as_float((unsigned)pv[q]), (int)(pv[q] >> 32));
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      am_take(best, bi, ob, oi);
    }
    if (j == 0) {
      if (bi == 0x7fffffff) bi = 0;  // all NaN (cannot happen with a sane model): torch.argmax -> 0
      const int64_t tok = fin ? (int64_t)sg.pad_id : (int64_t)bi;
      sg.ids[(int64_t)r * sg.ids_stride + L] = tok;
      const int done = fin || tok == sg.eos_id || (L + 1) >= sg.max_length;
      sg.unfinished[r] = done ? 0 : 1;
      n_unf += done ? 0 : 1;
    }
  }
  if (n_unf) atomicAdd(&am_nunf, n_unf);
  __syncthreads();
  if (tid == 0) {
    *sg.n_unfinished = am_nunf;
    __hip_atomic_store(sg.arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sg.cur_len = L + 1;
  }
}

template <bool AM>
__global__ __launch_bounds__(512) void lm_head_kernel(DecP p0, int groups_per_wg, LmGreedy sg) {
  DecP p = p0;  // blockIdx.z = 32-row chunk (beam rows), as in dec_linear_kernel
  p.M = min(32, p0.M - 32 * (int)blockIdx.z);
  p.x += (int64_t)32 * blockIdx.z * p0.ldx;
  if (p0.C) p.C = reinterpret_cast<float*>(p0.C) + (int64_t)32 * blockIdx.z * p0.ldc;
  __shared__ f32x4 red[3][MAXW][LMH_NCB][2][64];  // per-wave partial tiles, one slot per group in flight
  __shared__ float rpart[MAXW][32][2];
  __shared__ float rstat[32][2];
  __shared__ float econ[LMH_MAXG][LMH_NCB][2][16];  // [group][column block][colsum, bias][column]
  // the run's logits, written back after the loop as whole row spans: a group's 16 x 16 tiles stored in place were
  // 4 x 64-B pieces per wave instruction (rows 207 KB apart), 4 us of a 33 us launch (profiles/r05g_lmh_decomposition.txt)
  __shared__ float obuf[32][LMH_MAXG * LMH_NCB * 16 + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
  const int nkt = p.K >> 5;
  const int kt0 = (nkt * wave) / nw, kt1 = (nkt * (wave + 1)) / nw;  // <= LMH_KTM (host-checked)
  const int ktl = max(kt1 - 1, kt0);
  const int M = p.M;
  const int n_groups = (p.N + 16 * LMH_NCB - 1) / (16 * LMH_NCB);
  const int g0 = blockIdx.x * groups_per_wg, g1 = min(n_groups, g0 + groups_per_wg);
  if (g0 >= g1) return;
  // the run's weights through a bounds-checked buffer resource: a prefetch past the run (g >= g1) returns zeros
  // without a memory access, so every prefetch is unconditional (a conditional load made the compiler's wait counts
  // at the loop's joins assume it absent -- and wait for every load in flight).  The packed matrix pads N to 32
  // columns, so each of the run's groups has both column blocks.
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16x8*>(p.W) + (int64_t)g0 * LMH_NCB * nkt * 64, (short)0, (g1 - g0) * LMH_NCB * nkt * 1024, 0x00020000);
  auto wload = [&](int g, bf16x8 (&w)[LMH_NCB][LMH_KTM]) {
#pragma unroll
    for (int c = 0; c < LMH_NCB; ++c)
#pragma unroll
      for (int u = 0; u < LMH_KTM; ++u)
        w[c][u] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                   wrs, (((g - g0) * LMH_NCB + c) * nkt + min(kt0 + u, ktl)) * 1024 + lane * 16,
                                                   0, 2));  // aux 2 = nt
    __builtin_amdgcn_sched_barrier(0);  // the loads stay here, ahead of the waits for earlier groups
  };
  // issue order = wait order (vmcnt retires in order): the epilogue constants and the activation fragments first,
  // then the first two groups' weights, so the LayerNorm phase waits on the activations alone
  const int ncon = (g1 - g0) * LMH_NCB * 16;  // this run's columns: thread t stages columns t + j * blockDim
  float con_cs[LMH_ECJ], con_bn[LMH_ECJ];
  [[maybe_unused]] uint8_t con_mk[LMH_ECJ];
  [[maybe_unused]] int step_len = 0;
  __shared__ uint8_t smask[AM ? LMH_MAXG * LMH_NCB * 16 : 1];
#pragma unroll
  for (int j = 0; j < LMH_ECJ; ++j) {  // (clamped, not skipped: no load under a branch, host-checked coverage)
    const int t = min(tid + j * (int)blockDim.x, ncon - 1);
    const int n = min(g0 * LMH_NCB * 16 + t, p.N - 1);
    con_cs[j] = p.ln_colsum[n];
    con_bn[j] = p.bias ? p.bias[n] : 0.f;
    if constexpr (AM) con_mk[j] = sg.mask[n];
  }
  // AM: workgroup r < M scans row r's id history for EOS (stopping_criteria.py:75-77) while the weights stream --
  // wave 0, positions begin + lane + 64 u, loads clamped into the row (no wait on cur_len before issuing them)
  [[maybe_unused]] int row_fin = 0;
  [[maybe_unused]] int64_t hist[AM ? 7 : 1];
  if constexpr (AM) {
    step_len = *sg.cur_len;
    if ((int)blockIdx.x < M && wave == 0) {
      const int64_t* ids = sg.ids + (int64_t)blockIdx.x * sg.ids_stride;
#pragma unroll
      for (int u = 0; u < 7; ++u) hist[u] = ids[min(sg.begin_index + lane + 64 * u, (int)sg.ids_stride - 1)];
    }
  }
  // activation fragments of this wave's k-range, once (rows lane&15 and 16 + lane&15)
  bf16x8 a0[LMH_KTM], a1[LMH_KTM];
  {
    const int r0 = min(lane & 15, M - 1), r1 = min(16 + (lane & 15), M - 1), akoff = 8 * (lane >> 4);
#pragma unroll
    for (int u = 0; u < LMH_KTM; ++u) {
      const int k = min(kt0 + u, ktl) * 32 + akoff;
      a0[u] = *reinterpret_cast<const bf16x8*>(p.x + (int64_t)r0 * p.ldx + k);
      a1[u] = *reinterpret_cast<const bf16x8*>(p.x + (int64_t)r1 * p.ldx + k);
    }
  }
  bf16x8 wa[LMH_NCB][LMH_KTM], wb[LMH_NCB][LMH_KTM], wc[LMH_NCB][LMH_KTM];
  wload(g0, wa);
  wload(g0 + 1, wb);
#pragma unroll
  for (int j = 0; j < LMH_ECJ; ++j) {
    const int t = tid + j * (int)blockDim.x;
    if (t < ncon) {
      const int gi = t / (LMH_NCB * 16), c = (t / 16) % LMH_NCB, col = t % 16;
      econ[gi][c][0][col] = con_cs[j];
      econ[gi][c][1][col] = con_bn[j];
      if constexpr (AM) smask[t] = con_mk[j];
    }
  }
  // a wave with fewer than LMH_KTM k-tiles multiplies zero activations for the rest (exact: 0 x w adds +0), so the
  // loop's MFMAs carry no per-k-tile branch (whose joins made the compiler wait for every load in flight)
  bf16x8 za0[LMH_KTM], za1[LMH_KTM];
#pragma unroll
  for (int u = 0; u < LMH_KTM; ++u) {
    const bool in = kt0 + u < kt1;
    za0[u] = in ? a0[u] : bf16x8{};
    za1[u] = in ? a1[u] : bf16x8{};
  }
  // LayerNorm statistics of the 32 rows on the matrix cores (as dec_linear_kernel step 3)
  {
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
    f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0, q0 = s0, q1 = s0;
#pragma unroll
    for (int u = 0; u < LMH_KTM; ++u)
      if (kt0 + u < kt1) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], ones, s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], ones, s1, 0, 0, 0);
        q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], a0[u], q0, 0, 0, 0);
        q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], a1[u], q1, 0, 0, 0);
      }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        rpart[wave][4 * (lane >> 4) + i][0] = s0[i];
        rpart[wave][16 + 4 * (lane >> 4) + i][0] = s1[i];
      }
    }
    const int di = (lane & 15) - 4 * (lane >> 4);
    if (di >= 0 && di < 4) {
      rpart[wave][lane & 15][1] = q0[di];
      rpart[wave][16 + (lane & 15)][1] = q1[di];
    }
    __syncthreads();  // (also the epilogue constants: loaded before it)
    if (tid < 32) {
      float sx = 0.f, sq = 0.f;
      for (int w2 = 0; w2 < nw; ++w2) {
        sx += rpart[w2][tid][0];
        sq += rpart[w2][tid][1];
      }
      const float inv = 1.f / (float)p.K;
      const float mean = sx * inv;
      rstat[tid][0] = mean;
      rstat[tid][1] = rsqrtf(fmaxf(sq * inv - mean * mean, 0.f) + p.ln_eps);
    }
    __syncthreads();
  }
  // walk the run: groups g+1 and g+2 in flight while group g is multiplied, reduced and stored
  auto body = [&](int g, int slot, bf16x8 (&w)[LMH_NCB][LMH_KTM]) {
    f32x4 c0[LMH_NCB], c1[LMH_NCB];
#pragma unroll
    for (int c = 0; c < LMH_NCB; ++c) {
      c0[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      c1[c] = c0[c];
#pragma unroll
      for (int u = 0; u < LMH_KTM; ++u) {
        c0[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(za0[u], w[c][u], c0[c], 0, 0, 0);
        c1[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(za1[u], w[c][u], c1[c], 0, 0, 0);
      }
      red[slot][wave][c][0][lane] = c0[c];
      red[slot][wave][c][1][lane] = c1[c];
    }
    lmh_barrier();  // (three red slots: a slot is rewritten two barriers after its readers passed)
    // the 2 x NCB 16 x 16 tiles of the group, one per wave (a launch of fewer waves -- K < 640 -- takes several per
    // wave): wave-ordered sum, LayerNorm, bias, store
    for (int t = wave; t < 2 * LMH_NCB; t += nw) {
      const int c = t >> 1, hh = t & 1;
      f32x4 acc = red[slot][0][c][hh][lane];
      for (int w2 = 1; w2 < nw; ++w2) acc += red[slot][w2][c][hh][lane];
      const int n = (g * LMH_NCB + c) * 16 + (lane & 15);
      const float cs = econ[g - g0][c][0][lane & 15], bn = econ[g - g0][c][1][lane & 15];
      if (n < p.N) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * hh + 4 * (lane >> 4) + r;
          if (m < M) {
            obuf[m][(g - g0) * LMH_NCB * 16 + c * 16 + (lane & 15)] = rstat[m][1] * (acc[r] - rstat[m][0] * cs) + bn;
          }
        }
      }
    }
  };
  int g = g0;
  for (; g + 2 < g1; g += 3) {
    wload(g + 2, wc);
    body(g, 0, wa);
    wload(g + 3, wa);
    body(g + 1, 1, wb);
    wload(g + 4, wb);
    body(g + 2, 2, wc);
  }
  if (g < g1) body(g, 0, wa);
  if (g + 1 < g1) body(g + 1, 1, wb);
  // the run's logits: row m's columns [32 g0, 32 g1) as one contiguous span (each wave instruction 64 consecutive
  // floats = 256 B), non-temporal
  lmh_barrier();
  const int ncol = min(g1 * LMH_NCB * 16, p.N) - g0 * LMH_NCB * 16;
  if (p.C) {
    float* cbase = reinterpret_cast<float*>(p.C) + g0 * LMH_NCB * 16;
    for (int i = tid; i < M * ncol; i += blockDim.x) {
      const int m = i / ncol, col = i - m * ncol;
      __builtin_nontemporal_store(obuf[m][col], cbase + (int64_t)m * p.ldc + col);
    }
  }
  if constexpr (AM) {
    if ((int)blockIdx.x < M && wave == 0) {
      int f = 0;
#pragma unroll
      for (int u = 0; u < 7; ++u) f |= (sg.begin_index + lane + 64 * u < step_len && hist[u] == sg.eos_id) ? 1 : 0;
      row_fin = __builtin_amdgcn_ballot_w64(f != 0) != 0;
    }
    lm_greedy_tail(sg, obuf, smask, ncol, g0 * LMH_NCB * 16, M, step_len, row_fin);
  }
}

__global__ void pack_kernel(const bf16_t* __restrict__ W, int N, int K, bf16_t* __restrict__ out) {
  const int nkt = K >> 5;
  const int64_t total = (int64_t)((N + 31) / 32 * 2) * nkt * 64;
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

// Dynamic LDS of the activation image for a workgroup of ``tiles`` k-tiles (32 rows x (4 tiles + 1)
// 16-B chunks, rounded up to whole 1-KB LDS-DMA pieces).
size_t x_lds_bytes(int tiles) { return (size_t)((32 * (4 * tiles + 1) + 63) / 64) * 1024; }


// Launch geometry for (N, K): column blocks per workgroup, k-tiles per wave, waves, K splits.
struct Geo {
  int ncb, ktm, nw, ks;
};

Geo choose(int64_t N, int64_t K) {
  const int nkt = (int)(K / 32);
  const int blocks = (int)((N + 15) / 16);
  Geo g;
  g.ncb = blocks >= 320 ? 2 : 1;  // wide matrices: reuse each activation fragment twice
  g.ks = 1;
  // few columns, long K: split over workgroups, <= 27 k-tiles each (fc2 at large-v3: 6 splits; measured
  // 10.7 us vs 11.2 us for 8 splits and 13.0 us for 7 -- profiles/r01g_splitk_sweep.txt)
  if (blocks < 128 && nkt > 80) g.ks = (nkt + 26) / 27;
  const int per_wg0 = (nkt + g.ks - 1) / g.ks;
  // K <= 1280 without a split: 5 k-tiles per wave, up to 8 waves (more loads in flight per workgroup):
  // 1280x1280 5.8 -> 5.1 us, fc1 9.0 -> 8.6 us (profiles/r01h_declin_geo_sweep.txt); the LM head and
  // the split fc2 (6 x 27 k-tiles over 3 waves, r01g_splitk_sweep.txt) keep 10
  g.ktm = (g.ks == 1 && per_wg0 <= 40 && (N < 8192 || per_wg0 <= 5)) ? 5 : 10;  // (K <= 160: the u projection)
  // r04: the split fc2 (6 x 27 k-tiles) on 6 waves of 5 k-tiles instead of 3 of 10 -- more loads in flight per
  // workgroup: 9.79-9.89 vs 10.27-10.29 us (profiles/r04c_splitk_sweep.txt; ks 8 / 4 and the o-proj split worse)
  if (g.ks > 1 && per_wg0 <= 5 * MAXW && N < 8192) g.ktm = 5;
  const int per_wg = (nkt + g.ks - 1) / g.ks;
  g.nw = (per_wg + g.ktm - 1) / g.ktm;
  if (g.nw > MAXW) {  // very long K: more splits
    g.nw = MAXW;
    g.ks = (nkt + MAXW * g.ktm - 1) / (MAXW * g.ktm);
  }
  if (g.nw < 1) g.nw = 1;
  return g;
}

// LDS staging pays where one round of workgroups covers the grid (its 80-114 KB of LDS allows one
// workgroup per CU) and for the split-K workgroups (fc2: each stages its 32 rows x 864-element slice, 55 KB,
// two workgroups per CU: 10.3 vs 10.7 us, bitwise equal, profiles/r03_lab_notes.md r03y); the LM head's
// 1,621-workgroup grid keeps direct fragment loads at four workgroups per CU.
bool use_xlds(int64_t N, const Geo& g) { return g.ks > 1 || (N + 16 * g.ncb - 1) / (16 * g.ncb) <= 256; }
size_t x_lds_bytes_for(int nkt, int ks, bool xlds) { return xlds ? x_lds_bytes((nkt + ks - 1) / ks) : 0; }
// the image of a <= 16-row chunk (row split): only its rows' pieces are staged
size_t x_lds_bytes_rows(int tiles, int rows, bool xlds) {
  return xlds ? (size_t)((rows * (4 * tiles + 1) + 63) / 64) * 1024 : 0;
}

int device_cus() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  return ncu;
}

template <int KTM, int NCB, bool LNA, int EPI, typename TC, bool H2>
hipError_t launch_grid(const DecP& q, dim3 grid, dim3 block, size_t shm, int ks, hipStream_t s) {
  static size_t attr = 0;  // dynamic LDS this instantiation is cleared for
  if (shm > attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dec_linear_kernel<KTM, NCB, LNA, EPI, TC, H2>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    attr = shm;
  }
  hipLaunchKernelGGL((dec_linear_kernel<KTM, NCB, LNA, EPI, TC, H2>), grid, block, shm, s, q, ks);
  return hipGetLastError();
}

template <int KTM, int NCB, bool LNA, int EPI, typename TC>
hipError_t launch_one(const DecP& p, const Geo& g, hipStream_t s) {
  const int nkt = p.K / 32;
  if (g.ks == 1 && p.M > 32) {  // many rows: weight-stationary workgroups over row chunks
    const int ncg = (p.N + 16 * NCB - 1) / (16 * NCB), nz = (p.M + 31) / 32;
    const int zg0 = std::max(1, std::min(nz, (2 * device_cus()) / ncg));
    const int zper = (nz + zg0 - 1) / zg0, zg = (nz + zper - 1) / zper;
    hipLaunchKernelGGL((dec_linear_rows_kernel<KTM, NCB, LNA, EPI, TC>), dim3((unsigned)ncg, 1, (unsigned)zg),
                       dim3((unsigned)(64 * g.nw)), 0, s, p, zper);
    return hipGetLastError();
  }
  // row split: a grid whose doubled size still fits one round of one workgroup per CU (the 1280-column linears: 80
  // workgroups -> 160) runs its 17..32 rows as two 16-row chunks, each staging only its rows and computing one row
  // half (the H2 = false instantiation), every output element by the same operations (rows are independent):
  // bitwise the 32-row launch.  o 5.05 -> 4.13-4.29 us; fc1 (160 -> 320 workgroups, two per CU) measured
  // 8.6 -> 8.7-8.9 us, so it keeps one launch of 32-row tiles (profiles/r04o_rowsplit_ab.txt)
  const int ncg = (p.N + 16 * NCB - 1) / (16 * NCB);
  const bool split = g.ks == 1 && p.M > 16 && p.M <= 32 && 2 * ncg <= device_cus();
  DecP q = p;
  q.zrows = split ? 16 : 32;
  const dim3 grid((unsigned)ncg, (unsigned)g.ks, (unsigned)((p.M + q.zrows - 1) / q.zrows));
  const dim3 block((unsigned)(64 * g.nw));
  if (split) return launch_grid<KTM, NCB, LNA, EPI, TC, false>(q, grid, block, x_lds_bytes_rows((nkt + g.ks - 1) / g.ks, 16, p.xlds), g.ks, s);
  return launch_grid<KTM, NCB, LNA, EPI, TC, true>(q, grid, block, x_lds_bytes_for(nkt, g.ks, p.xlds), g.ks, s);
}

template <int KTM, int NCB>
hipError_t launch_k(const DecP& p, bool resid, const Geo& g, bool c_f32, hipStream_t s) {
  if (resid) return launch_one<KTM, NCB, false, KW_EPI_RESID, float>(p, g, s);  // (no LayerNorm-fused residual linear)
  if (p.ln)
    return c_f32 ? launch_one<KTM, NCB, true, KW_EPI_STORE, float>(p, g, s) : launch_one<KTM, NCB, true, KW_EPI_STORE, bf16_t>(p, g, s);
  return c_f32 ? launch_one<KTM, NCB, false, KW_EPI_STORE, float>(p, g, s) : launch_one<KTM, NCB, false, KW_EPI_STORE, bf16_t>(p, g, s);
}

hipError_t launch(const DecP& p, bool resid, const Geo& g, bool c_f32, hipStream_t s) {
  if (g.ktm == 5) return g.ncb == 2 ? launch_k<5, 2>(p, resid, g, c_f32, s) : launch_k<5, 1>(p, resid, g, c_f32, s);
  return g.ncb == 2 ? launch_k<10, 2>(p, resid, g, c_f32, s) : launch_k<10, 1>(p, resid, g, c_f32, s);
}

// the LM head's column groups per workgroup: one run per CU
int lmh_groups_per_wg(int64_t N) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  const int groups = (int)((N + 16 * LMH_NCB - 1) / (16 * LMH_NCB));
  return (groups + ncu - 1) / ncu;
}

// the persistent LM head (lm_head_kernel) covers the shape: <= 8 waves of LMH_KTM k-tiles, <= LMH_MAXG groups per
// workgroup, the run's epilogue constants staged by one pass of LMH_ECJ per thread
bool lmh_fits(int64_t M, int64_t N, int nkt) {
  const int per = lmh_groups_per_wg(N);
  return (nkt + LMH_KTM - 1) / LMH_KTM <= MAXW && M <= LMH_MAX_ROWS && per <= LMH_MAXG &&
         64 * ((nkt + LMH_KTM - 1) / LMH_KTM) * LMH_ECJ >= per * LMH_NCB * 16;
}

// kw_dec_lm_greedy's grid (one run of column groups per workgroup, as kw_dec_linear's LM head)
int lmg_grid(int64_t N) {
  const int groups = (int)((N + 16 * LMH_NCB - 1) / (16 * LMH_NCB)), per = lmh_groups_per_wg(N);
  return (groups + per - 1) / per;
}
constexpr int LMG_MAXG = 256;  // workgroups whose partials the last arriver merges (16 per lane)

}  // namespace

extern "C" size_t kw_dec_lm_greedy_workspace(int64_t B, int64_t V) {
  const int64_t groups = (V + 16 * LMH_NCB - 1) / (16 * LMH_NCB);  // >= the grid on any device
  return 256 + (size_t)B * (size_t)std::min<int64_t>(groups, LMG_MAXG) * sizeof(unsigned long long);
}

extern "C" int kw_dec_lm_greedy_supported(int64_t B, int64_t V, int64_t d) {
  return B >= 1 && B <= LMH_MAX_ROWS && V >= 8192 && d > 0 && d % 32 == 0 && lmh_fits(B, V, (int)(d / 32)) &&
                 lmg_grid(V) <= LMG_MAXG
             ? 1
             : 0;
}

extern "C" int kw_dec_lm_greedy(const kw_dec_linear_args* a, const kw_sampler_args* g, kw_stream_t stream) {
  if (!a || !g || !a->x || !a->W || !a->ln || !a->ln_colsum || a->K <= 0 || a->K % 32 != 0 || a->ldx % 8 != 0 ||
      a->ldx < a->K || (uintptr_t)a->x % 16 != 0 || a->epilogue != KW_EPI_STORE || a->gelu || a->scale_cols != 0 ||
      (a->C && (a->c_dtype != KW_DT_F32 || a->ldc < a->N)))
    return kw_set_error_msg(KW_EINVAL, "kw_dec_lm_greedy: the LM head must be LayerNorm-fused STORE into f32 (or no) logits");
  if (!g->suppress_mask || !g->ids || !g->cur_len || !g->unfinished || !g->n_unfinished || !g->workspace ||
      (g->n_begin_suppress > 0 && !g->begin_suppress) || g->B != a->M || g->V != a->N)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_lm_greedy: sampler arguments missing or not the LM head's B x V");
  if (g->return_timestamps || g->scores_out)
    return kw_set_error_msg(KW_EUNSUPPORTED, "kw_dec_lm_greedy: no timestamps, no scores_out (use kw_greedy_step)");
  if (!kw_dec_lm_greedy_supported(a->M, a->N, a->K))
    return kw_set_error_msg(KW_EUNSUPPORTED, "kw_dec_lm_greedy: shape not covered (kw_dec_lm_greedy_supported)");
  if (g->ws_bytes < kw_dec_lm_greedy_workspace(a->M, a->N) || (uintptr_t)g->workspace % 16 != 0)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_lm_greedy: needs a zero-filled workspace of kw_dec_lm_greedy_workspace()");
  DecP p{};
  p.x = reinterpret_cast<const bf16_t*>(a->x);
  p.ldx = a->ldx;
  p.ln = 1;
  p.ln_eps = a->ln_eps;
  p.ln_colsum = a->ln_colsum;
  p.W = reinterpret_cast<const bf16x8*>(a->W);
  p.bias = a->bias;
  p.C = a->C;
  p.ldc = a->ldc;
  p.M = (int)a->M;
  p.N = (int)a->N;
  p.K = (int)a->K;
  LmGreedy sg{};
  sg.mask = g->suppress_mask;
  sg.bsup = g->begin_suppress;
  sg.nbsup = g->n_begin_suppress;
  sg.ids = g->ids;
  sg.ids_stride = g->ids_stride;
  sg.cur_len = g->cur_len;
  sg.max_length = g->max_length;
  sg.begin_index = g->begin_index;
  sg.eos_id = g->eos_id;
  sg.pad_id = g->pad_id;
  sg.unfinished = g->unfinished;
  sg.n_unfinished = g->n_unfinished;
  sg.arrive = reinterpret_cast<int*>(g->workspace);
  sg.fin = reinterpret_cast<int*>(g->workspace) + 32;
  sg.part = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(g->workspace) + 256);
  const int nkt = (int)(a->K / 32), nwv = (nkt + LMH_KTM - 1) / LMH_KTM;
  hipLaunchKernelGGL(lm_head_kernel<true>, dim3((unsigned)lmg_grid(a->N)), dim3((unsigned)(64 * nwv)), 0,
                     (hipStream_t)stream, p, lmh_groups_per_wg(a->N), sg);
  KW_CHECK_LAUNCH();
  return KW_OK;
}

extern "C" size_t kw_dec_linear_workspace_bytes(int64_t N, int64_t K) {
  const Geo g = choose(N, K);
  const int64_t ncg = (N + 16 * g.ncb - 1) / (16 * g.ncb);
  return (size_t)CNT_MAX * sizeof(int) + (g.ks > 1 ? (size_t)ZMAX * ncg * g.ks * g.ncb * 512 * sizeof(float) : 0);
}

extern "C" int kw_dec_linear(const kw_dec_linear_args* a, kw_stream_t stream) {
  if (!a || !a->x || !a->W || a->M < 0 || a->N <= 0 || a->K <= 0 || a->K % 32 != 0 || a->ldx % 8 != 0 || a->ldx < a->K ||
      (uintptr_t)a->x % 16 != 0)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_linear: null pointer or bad sizes (K % 32 == 0, ldx % 8 == 0, x 16-B aligned)");
  if (a->epilogue == KW_EPI_RESID) {
    if (!a->h || !a->hb || a->ldh < a->N)
      return kw_set_error_msg(KW_EINVAL, "kw_dec_linear: RESID needs h (f32) and hb (bf16) with ldh >= N");
  } else if (a->epilogue == KW_EPI_STORE) {
    if (!a->C || a->ldc < a->N || (a->c_dtype != KW_DT_F32 && a->c_dtype != KW_DT_BF16))
      return kw_set_error_msg(KW_EINVAL, "kw_dec_linear: STORE needs C (f32 or bf16) with ldc >= N");
  } else {
    return kw_set_error_msg(KW_EINVAL, "kw_dec_linear: epilogue must be STORE or RESID");
  }
  if (a->ln && (!a->ln_colsum || a->epilogue != KW_EPI_STORE))
    return kw_set_error_msg(KW_EINVAL, "kw_dec_linear: fused LayerNorm needs ln_colsum and the STORE epilogue");
  if (a->M == 0) return KW_OK;
  const Geo g = choose(a->N, a->K);
  const int nkt = (int)(a->K / 32);
  if ((nkt + g.ks * g.nw - 1) / (g.ks * g.nw) > g.ktm || g.ks > KSMAX || (a->ln && g.ks > 1))
    return kw_set_error_msg(KW_EUNSUPPORTED, "kw_dec_linear: K too long for the k-tile budget");
  const int64_t ncg = (a->N + 16 * g.ncb - 1) / (16 * g.ncb);
  if (g.ks > 1) {
    if (ncg * ZMAX > CNT_MAX) return kw_set_error_msg(KW_EINVAL, "kw_dec_linear: split-K needs N <= 8192");
    if (!a->workspace || a->ws_bytes < kw_dec_linear_workspace_bytes(a->N, a->K))
      return kw_set_error_msg(KW_EINVAL, "kw_dec_linear: needs a zero-filled workspace of kw_dec_linear_workspace_bytes()");
  }
  hipStream_t s = (hipStream_t)stream;
  // LM head: LayerNorm-fused, f32 logits, a wide N and a short K -> the persistent weight stream up to
  // 32 rows, the all-rows GEMM up to LMR_MAXROWS (beam rows), the weight-stationary rows kernel beyond
  const bool lm_shape = a->ln && a->epilogue == KW_EPI_STORE && a->c_dtype == KW_DT_F32 && a->N >= 8192 && !a->gelu &&
                        a->scale_cols == 0;
  if (lm_shape && a->M > LMH_MAX_ROWS && a->M <= LMR_MAXROWS && nkt % 8 == 0) {
    DecP p{};
    p.x = reinterpret_cast<const bf16_t*>(a->x);
    p.ldx = a->ldx;
    p.ln = 1;
    p.ln_eps = a->ln_eps;
    p.ln_colsum = a->ln_colsum;
    p.W = reinterpret_cast<const bf16x8*>(a->W);
    p.bias = a->bias;
    p.C = a->C;
    p.ldc = a->ldc;
    p.M = (int)a->M;
    p.N = (int)a->N;
    p.K = (int)a->K;
    const int n_cb = (int)((a->N + 15) / 16);
    // eight 16-column waves per workgroup, four k-tile slices staged ahead (one workgroup per CU); a slice holds
    // 128 G rows, G = ceil(M / 128)
    const dim3 grid((unsigned)((n_cb + 7) / 8));
    switch ((a->M + 127) / 128) {
      case 1: hipLaunchKernelGGL((lm_head_rows_kernel<8, 1, 4>), grid, dim3(512), 0, s, p); break;
      case 2: hipLaunchKernelGGL((lm_head_rows_kernel<8, 2, 8>), grid, dim3(512), 0, s, p); break;
      default: hipLaunchKernelGGL((lm_head_rows_kernel<8, 3, LMR_NZ>), grid, dim3(512), 0, s, p); break;
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? KW_OK : kw_set_error(e);
  }
  const bool lmh = lm_shape && lmh_fits(a->M, a->N, nkt);
  // rows: one launch with a grid z-slice per 32-row chunk (K-split launches: up to ZMAX chunks each)
  const int64_t step = (g.ks == 1 || lmh) ? a->M : 32 * ZMAX;
  for (int64_t m0 = 0; m0 < a->M; m0 += step) {
    DecP p;
    p.M = (int)(a->M - m0 < step ? a->M - m0 : step);
    p.N = (int)a->N;
    p.K = (int)a->K;
    p.x = reinterpret_cast<const bf16_t*>(a->x) + m0 * a->ldx;
    p.ldx = a->ldx;
    p.ln = a->ln;
    p.ln_eps = a->ln_eps;
    p.ln_colsum = a->ln_colsum;
    p.W = reinterpret_cast<const bf16x8*>(a->W);
    p.bias = a->bias;
    const size_t csz = a->c_dtype == KW_DT_F32 ? 4 : 2;
    p.C = a->C ? reinterpret_cast<char*>(a->C) + m0 * a->ldc * csz : nullptr;
    p.ldc = a->ldc;
    p.gelu = a->gelu;
    p.scale = a->scale;
    p.scale_cols = (int)a->scale_cols;
    p.h = a->h ? a->h + m0 * a->ldh : nullptr;
    p.hb = a->hb ? reinterpret_cast<bf16_t*>(a->hb) + m0 * a->ldh : nullptr;
    p.ldh = a->ldh;
    p.cnt = reinterpret_cast<int*>(a->workspace);
    p.slab = a->workspace ? reinterpret_cast<float*>(reinterpret_cast<char*>(a->workspace) + CNT_MAX * sizeof(int)) : nullptr;
    p.xlds = use_xlds(a->N, g) ? 1 : 0;
    // 16-B epilogue pieces: whole 16-column blocks and 16-B aligned rows (every z-chunk's rows too)
    p.vec_epi = a->N % 16 == 0 &&
                (a->epilogue == KW_EPI_RESID
                     ? a->ldh % 8 == 0 && (uintptr_t)p.h % 16 == 0 && (uintptr_t)p.hb % 16 == 0
                     : (a->ldc * (int64_t)csz) % 16 == 0 && (uintptr_t)p.C % 16 == 0);
    if (lmh) {
      const int groups = (int)((a->N + 16 * LMH_NCB - 1) / (16 * LMH_NCB));
      const int per = lmh_groups_per_wg(a->N);
      const int nwv = (nkt + LMH_KTM - 1) / LMH_KTM;
      hipLaunchKernelGGL(lm_head_kernel<false>, dim3((unsigned)((groups + per - 1) / per), 1, (unsigned)((p.M + 31) / 32)),
                         dim3((unsigned)(64 * nwv)), 0, s, p, per, LmGreedy{});
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return kw_set_error(e);
      continue;
    }
    hipError_t e = launch(p, a->epilogue == KW_EPI_RESID, g, a->c_dtype == KW_DT_F32, s);
    if (e != hipSuccess) return kw_set_error(e);
  }
  return KW_OK;
}

extern "C" size_t kw_packed_weight_bytes(int64_t N, int64_t K) { return (size_t)((N + 31) / 32) * 32 * (size_t)K * 2; }

extern "C" int kw_pack_weight(const void* W, int64_t N, int64_t K, void* packed, kw_stream_t stream) {
  if (!W || !packed || N <= 0 || K <= 0 || K % 32 != 0)
    return kw_set_error_msg(KW_EINVAL, "kw_pack_weight: needs K % 32 == 0");
  hipLaunchKernelGGL(pack_kernel, dim3(1024), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)W, (int)N, (int)K,
                     (bf16_t*)packed);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
