// Attention kernels for the Whisper hot path on gfx950.
//
// Encoder (K6): flash-style bf16 attention, non-causal, T = 1500, head_dim 64
// (TF/models/whisper/modeling_whisper.py:284-356 + TF/integrations/sdpa_attention.py:79-166;
// q arrives pre-scaled by head_dim^-0.5 from the QKV epilogue, modeling_whisper.py:309).
//   Per workgroup: one (batch, head, 128-query tile); 4 waves x 32 queries.  Scores are computed
//   TRANSPOSED, S^T = K Q^T (v_mfma_f32_32x32x16_bf16), so each lane owns one query's scores and the
//   row softmax needs only in-lane math plus one lane^32 exchange.  O^T = V^T P^T takes P^T straight
//   from the S^T accumulators (no LDS round trip) and V^T from a row-major V tile through
//   ds_read_b64_tr_b16.  K/V tiles (64 keys) are staged global->LDS by global_load_lds_dwordx4 into a
//   2-deep ring with XOR-swizzled images (K: chunk ^ ((row>>1)&7) for ds_read_b128; V: chunk ^
//   (((row>>1)&1)<<2) for the transposed reads) -- both conflict-free.  O is normalised and staged
//   through LDS for 16-B coalesced stores.
// Encoder f32 path: exact-fp32 reference-order kernel for the parity mode.
// Decoder self-attention (K10): static KV cache append + attention; one new position per row splits
//   the keys into <= 256-key chunks like the cross-attention (prefill, q_len > 1: one workgroup per
//   (b, h) walking the queries).
// Decoder cross-attention (K11): split-S partial softmax over cached encoder K/V in <= 256-key chunks,
//   8 lanes per key row so every K and V load is a coalesced 1-KB wave access, and every load of the
//   chunk (64 KB) issued before the first score; the last-arriving chunk combines the partials in the
//   same launch (write-through partials + arrival counter, MI355X_MICROARCH "Valid forms" row 1).
#include <math.h>

#include "attn_common.h"
#include "decproj.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(2))) unsigned int v2u32;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u32;

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

namespace {


__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// lane ^ 32 reductions by v_permlane32_swap (a VALU half-exchange; no LDS round trip like ds_bpermute):
// with both operands = v, one result holds the lane's own value and the other its partner's
__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ------------------------------------------------------------------------------------------------
// encoder flash attention, bf16
// ------------------------------------------------------------------------------------------------
constexpr int AQ = 128;        // queries per workgroup
constexpr int AK = 64;         // keys per tile
constexpr int TILE_BYTES = AK * HD * 2;  // 8 KB
constexpr int ATT_LDS = 2 * 2 * TILE_BYTES;  // K,V x 2 stages = 32 KB (O staging reuses it)

__global__ __launch_bounds__(256, 2) void attn_fwd_bf16(const bf16_t* __restrict__ qkv, int B, int H, int T,
                                                       bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char smem[ATT_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_qt = (T + AQ - 1) / AQ;
  const int bh = blockIdx.x / n_qt;
  const int qt = blockIdx.x - bh * n_qt;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int64_t head_elems = (int64_t)T * HD;
  const bf16_t* Q = qkv + ((int64_t)(0 * B + b) * H + h) * head_elems;
  const bf16_t* K = qkv + ((int64_t)(1 * B + b) * H + h) * head_elems;
  const bf16_t* V = qkv + ((int64_t)(2 * B + b) * H + h) * head_elems;

  const int q_lane = qt * AQ + wave * 32 + (lane & 31);
  const int hh = lane >> 5;
  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16s + 8h .. +7]
  bf16x8 qf[4];
  {
    const int qr = min(q_lane, T - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)qr * HD + 16 * s + 8 * hh);
  }

  // staging: each tile (64 rows x 128 B) = 8 glds instructions; wave w issues rows [16w, 16w+16)
  const int n_kt = (T + AK - 1) / AK;
  auto stage = [&](int s, int kt) {
    char* kb = smem + s * 2 * TILE_BYTES;
    char* vb = kb + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int g = wave * 2 + i;  // 8-row group
      const int row = 8 * g + (lane >> 3);
      const int key = min(kt * AK + row, T - 1);
      const int slot = lane & 7;
      const int ck = slot ^ ((row >> 1) & 7);
      const int cv = slot ^ (((row >> 1) & 1) << 2);
      glds16(K + (int64_t)key * HD + ck * 8, kb + g * 1024);
      glds16(V + (int64_t)key * HD + cv * 8, vb + g * 1024);
    }
  };

  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  stage(0, 0);
  for (int kt = 0; kt < n_kt; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < n_kt) stage((kt + 1) & 1, kt + 1);
    const char* kb = smem + (kt & 1) * 2 * TILE_BYTES;
    const char* vb = kb + TILE_BYTES;

    // S^T for 2 key blocks of 32
    f32x16 st[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[i][r] = 0.f;
      const int row = i * 32 + (lane & 31);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int c = 2 * s + hh;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
        st[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st[i], 0, 0, 0);
      }
    }
    // mask keys >= T (last tile only), row max
    const int key0 = kt * AK;
    if (key0 + AK > T) {  // ragged last tile only
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = key0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key >= T) st[i][r] = -INFINITY;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[i][r]);
    mx = xor32_max(mx);
    float rs = 0.f;
    bf16x8 pf[2][2];
    {
      // deferred rescale: the exponent reference m_run only moves when a score exceeds it by more than
      // 8 (p <= e^8, exact in f32 and in bf16's range); most tiles skip the O / l rescale entirely
      const bool bump = mx > m_run + 8.0f;
      if (__builtin_amdgcn_ballot_w64(bump)) {
        const float m_new = bump ? mx : m_run;
        const float alpha = bump ? __builtin_amdgcn_exp2f((m_run - m_new) * LOG2E) : 1.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
        l_run *= alpha;
        m_run = m_new;
      }
      const float mneg = -m_run * LOG2E;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            // raw v_exp_f32: arguments are <= 8 * log2(e) and very negative ones may flush to 0
            const float p = __builtin_amdgcn_exp2f(fmaf(st[i][8 * s + e], LOG2E, mneg));
            rs += p;
            pf[i][s][e] = (__bf16)p;
          }
    }
    l_run += xor32_sum(rs);

    // O^T += V^T P^T ; A operand via ds_read_b64_tr_b16 from the row-major V tile.  The transposed
    // reads are inline asm: as builtins the compiler cannot tell the V image from the next tile's
    // in-flight LDS-DMA and puts an s_waitcnt vmcnt(0) (wait for the prefetch) in front of them.
    // Step n = (key block i, 16-key step s) reads 4 pieces; step n+1's reads are issued before step
    // n's MFMAs (counted lgkmcnt).
    const int li = lane & 15, qq = li >> 2, pp = li & 3, grp = (lane >> 4) & 1;
    auto vread = [&](int n, v2u32 (&t)[2][2]) {
      const int i = n >> 1, s = n & 1;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int row = i * 32 + 16 * s + 8 * half + 4 * hh + qq;
          const int chunk = db * 4 + 2 * grp + (pp >> 1);
          const int off = row * 128 + ((chunk ^ (((row >> 1) & 1) << 2)) << 4) + (pp & 1) * 8;
          asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(t[db][half]) : "v"(lds_u32(vb + off)));
        }
    };
    v2u32 vt[2][2][2];
    vread(0, vt[0]);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      if (n + 1 < 4) {
        vread(n + 1, vt[(n + 1) & 1]);
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(vt[n & 1][0][0]), "+v"(vt[n & 1][0][1]), "+v"(vt[n & 1][1][0]),
                     "+v"(vt[n & 1][1][1]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vt[n & 1][0][0]), "+v"(vt[n & 1][0][1]), "+v"(vt[n & 1][1][0]),
                     "+v"(vt[n & 1][1][1]));
      }
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const v4u32 w = {vt[n & 1][db][0][0], vt[n & 1][db][0][1], vt[n & 1][db][1][0], vt[n & 1][db][1][1]};
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[n >> 1][n & 1], o[db], 0, 0, 0);
      }
    }
  }

  // normalise and stage O (q rows x 64 hd, bf16) through LDS for coalesced stores
  __syncthreads();
  bf16_t* os = reinterpret_cast<bf16_t*>(smem) + wave * 32 * HD;  // 4 KB per wave
  const float inv_l = 1.0f / l_run;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = db * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      os[(lane & 31) * HD + d] = f2bf(o[db][r] * inv_l);
    }
  __syncthreads();
  // each wave writes its 32 rows x 128 B: 256 16-B chunks, 4 per lane
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int chunk = i * 64 + lane;
    const int qr = chunk >> 3, cc = chunk & 7;
    const int q = qt * AQ + wave * 32 + qr;
    if (q < T) {
      const uint4 v = *reinterpret_cast<const uint4*>(os + qr * HD + cc * 8);
      *reinterpret_cast<uint4*>(out + ((int64_t)b * T + q) * (H * HD) + h * HD + cc * 8) = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Encoder attention with log2-unit q (the bf16 engine, kw_attention's KW_ATTN_Q_LOG2).  q carries log2(e) too
// (folded into the QKV GEMM epilogue's q scale: one bf16 rounding as before) and the matrix cores subtract the
// running reference: a fifth k-step per 32-key block multiplies K~ = (1, 1, 0, ...) by Q~ = (hi, lo, 0, ...) with
// hi + lo = -m_run (two bf16 terms: exact to 2^-16 of m_run), so the MFMA output is already the exponent and
// p = exp2(s) is ONE v_exp per score.  The reference moves only when a score exceeds it by more than 8 / ln 2
// (p <= e^8), then that tile is shifted once more and O / l rescaled.  The kernel is vector-issue-bound (18 MFMAs
// per 64-key tile beside 32 v_exp, the row sums and the bf16 packing), so the tile does nothing else:
//  * no row maximum on the common path: the tile's p = exp2(s) and row sums are computed straight away; only a
//    wave in which some lane's sum exceeds 2980 (< e^8 = 2^11.5415602: a lane whose maximum would move the
//    reference has a p, hence a sum, above it; NaN takes the branch too) computes the maxima, moves the
//    reference and recomputes the tile (its scores again from the same LDS image: bitwise) -- every lane ends
//    with the p of the always-compute-the-maximum order (r03x: bitwise equal to that kernel on every shape
//    tested, 405 vs 460 us per launch at large-v3 B = 32, tools/lab/enc_attn_l2_ab.py);
//  * the two ring stages as static parities (the loop unrolled by two): every LDS fragment read is a lane base
//    plus an immediate offset;
//  * K / V tiles by buffer_load ... lds from per-head buffer descriptors (base and size in SGPRs, advanced per
//    tile on the scalar unit): no per-tile address arithmetic, and rows past T read as zeros (the ragged last
//    tile's scores there are masked to -inf; their V rows enter as 0 * 0).
// (Row sums as P.1 on the matrix cores: 143 registers, 3 waves per SIMD, slower -- profiles/r03_lab_notes.md)
template <int N_, int PAR>  // one 16-key step of the P.V product: V^T fragments by transposed reads at immediates
__device__ __forceinline__ void attn_vread(uint32_t b0, uint32_t b1, v2u32 (&t)[2][2]) {
  constexpr int i = N_ >> 1, s = N_ & 1;
  constexpr int o0 = PAR * 2 * TILE_BYTES + TILE_BYTES + (i * 32 + 16 * s) * 128;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(t[0][0]) : "v"(b0), "i"(o0));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(t[0][1]) : "v"(b0), "i"(o0 + 8 * 128));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(t[1][0]) : "v"(b1), "i"(o0));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(t[1][1]) : "v"(b1), "i"(o0 + 8 * 128));
}

__global__ __launch_bounds__(256, 4) void attn_fwd_l2(const bf16_t* __restrict__ qkv, int B, int H, int T,
                                                      bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char smem[ATT_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_qt = (T + AQ - 1) / AQ;
  const int bh = blockIdx.x / n_qt;
  const int qt = blockIdx.x - bh * n_qt;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int64_t head_elems = (int64_t)T * HD;
  const bf16_t* Q = qkv + ((int64_t)(0 * B + b) * H + h) * head_elems;
  const bf16_t* K = qkv + ((int64_t)(1 * B + b) * H + h) * head_elems;
  const bf16_t* V = qkv + ((int64_t)(2 * B + b) * H + h) * head_elems;

  const int q_lane = qt * AQ + wave * 32 + (lane & 31);
  const int hh = lane >> 5;
  bf16x8 qf[4];
  {
    const int qr = min(q_lane, T - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)qr * HD + 16 * s + 8 * hh);
  }

  // staging (attn_fwd_bf16's image): wave w moves rows [16w, 16w + 16) of each tile, lane = (row, 16-B slot)
  uint32_t voff_k[2], voff_v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (wave * 2 + i) + (lane >> 3);
    const int slot = lane & 7;
    voff_k[i] = (uint32_t)(row * HD + (slot ^ ((row >> 1) & 7)) * 8) * 2;
    voff_v[i] = (uint32_t)(row * HD + (slot ^ (((row >> 1) & 1) << 2)) * 8) * 2;
  }
  const int n_kt = (T + AK - 1) / AK;
  if (T % AK) {  // rows past T: whatever the DMA leaves there must be finite (their P is 0; 0 * NaN is not)
#pragma unroll
    for (int i = 0; i < ATT_LDS / (256 * 16); ++i)
      *reinterpret_cast<uint4*>(smem + (i * 256 + tid) * 16) = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }
  auto stage = [&](auto par_c, int kt) __attribute__((always_inline)) {
    constexpr int par = decltype(par_c)::value;
    const int nrec = (T - kt * AK) * HD * 2;  // this tile's rows to the head's end: later rows read as 0
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)(K + (int64_t)kt * AK * HD), (short)0, nrec, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)(V + (int64_t)kt * AK * HD), (short)0, nrec, 0x00020000);
    char* kb = smem + par * 2 * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int g = wave * 2 + i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)(kb + g * 1024), 16, voff_k[i], 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(kb + TILE_BYTES + g * 1024), 16,
                                               voff_v[i], 0, 0, 0);
    }
  };

  // fragment-read lane bases: K rows (lane & 31) + 32 i, 16-B chunk (2 s + hh) ^ ((row >> 1) & 7) per k-step s;
  // V^T by transposed reads, 16-B chunk (db ^ ((qq >> 1) & 1)) * 4 + 2 grp + (pp >> 1) (attn_fwd_bf16's vread)
  const uint32_t sbase = lds_u32(smem);
  uint32_t kofs[4];
  {
    const int r = lane & 31, r7 = (r >> 1) & 7;
#pragma unroll
    for (int s = 0; s < 4; ++s) kofs[s] = (uint32_t)(r * 128 + (((2 * s + hh) ^ r7) << 4));
  }
  uint32_t vb0, vb1;
  {
    const int li = lane & 15, qq = li >> 2, pp = li & 3, grp = (lane >> 4) & 1, x = (qq >> 1) & 1;
    const uint32_t lanepart = (uint32_t)((4 * hh + qq) * 128 + (2 * grp + (pp >> 1)) * 16 + (pp & 1) * 8);
    vb0 = sbase + lanepart + (uint32_t)((0 ^ x) * 64);
    vb1 = sbase + lanepart + (uint32_t)((1 ^ x) * 64);
  }

  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = 0.f, l_run = 0.f;
  bf16x8 kone, qref;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    kone[e] = (__bf16)((hh == 0 && e < 2) ? 1.0f : 0.0f);
    qref[e] = (__bf16)0.0f;
  }

  auto tile = [&](auto par_c, auto first_c, int kt) __attribute__((always_inline)) {
    constexpr int par = decltype(par_c)::value;
    constexpr bool first = decltype(first_c)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < n_kt) stage(std::integral_constant<int, 1 - par>{}, kt + 1);
    const char* kb = smem + par * 2 * TILE_BYTES;

    // S^T for 2 key blocks of 32 (log2 units, minus the reference), keys >= T masked in the ragged last tile
    f32x16 st[2];
    auto scores = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) st[i][r] = 0.f;
        st[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kone, qref, st[i], 0, 0, 0);  // -m_run
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + i * 32 * 128 + kofs[s]);
          st[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st[i], 0, 0, 0);
        }
      }
      const int key0 = kt * AK;
      if (key0 + AK > T) {  // ragged last tile only
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = key0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key >= T) st[i][r] = -INFINITY;
          }
      }
    };
    scores();
    float rs;
    bf16x8 pf[2][2];
    auto expsum = [&]() __attribute__((always_inline)) {
      rs = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float p = __builtin_amdgcn_exp2f(st[i][8 * s + e]);
            rs += p;
            pf[i][s][e] = (__bf16)p;
          }
    };
    // the reference move: only where a score exceeds the reference by more than 8 / ln 2
    auto rebase = [&]() __attribute__((always_inline)) {
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[i][r]);
      mx = xor32_max(mx);
      const bool bump = first || mx > 11.5415602f;
      if (__builtin_amdgcn_ballot_w64(bump)) {
        const float d = bump ? mx : 0.f;
        const float alpha = (bump && !first) ? __builtin_amdgcn_exp2f(-d) : 1.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            o[i][r] *= alpha;
            st[i][r] -= d;
          }
        l_run *= alpha;
        m_run += d;
        const float nm = -m_run;
        const __bf16 hi = (__bf16)nm;
        const __bf16 lo = (__bf16)(nm - (float)hi);
        qref[0] = hh == 0 ? hi : (__bf16)0.0f;
        qref[1] = hh == 0 ? lo : (__bf16)0.0f;
      }
    };
    if constexpr (first) {
      rebase();
      expsum();
    } else {
      expsum();
      if (__builtin_amdgcn_ballot_w64(!(rs <= 2980.0f))) {  // rare: some lane may move its reference
        // the scores again (the same MFMAs on the same LDS image: bitwise), so st need not stay live through the
        // common path (opaque operands: the compiler would otherwise keep the first st instead)
        asm volatile("" : "+v"(qref), "+v"(kone)::"memory");
        scores();
        rebase();
        expsum();
      }
    }
    l_run += xor32_sum(rs);

    // O^T += V^T P^T (attn_fwd_bf16's order): step n + 1's transposed reads issued before step n's MFMAs
    v2u32 vt[2][2][2];
    attn_vread<0, par>(vb0, vb1, vt[0]);
    auto pv = [&](auto n_c) __attribute__((always_inline)) {
      constexpr int n = decltype(n_c)::value;
      if constexpr (n + 1 < 4) {
        attn_vread<n + 1, par>(vb0, vb1, vt[(n + 1) & 1]);
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(vt[n & 1][0][0]), "+v"(vt[n & 1][0][1]), "+v"(vt[n & 1][1][0]),
                     "+v"(vt[n & 1][1][1]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vt[n & 1][0][0]), "+v"(vt[n & 1][0][1]), "+v"(vt[n & 1][1][0]),
                     "+v"(vt[n & 1][1][1]));
      }
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const v4u32 w = {vt[n & 1][db][0][0], vt[n & 1][db][0][1], vt[n & 1][db][1][0], vt[n & 1][db][1][1]};
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[n >> 1][n & 1], o[db], 0, 0, 0);
      }
    };
    pv(std::integral_constant<int, 0>{});
    pv(std::integral_constant<int, 1>{});
    pv(std::integral_constant<int, 2>{});
    pv(std::integral_constant<int, 3>{});
  };

  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using F = std::integral_constant<bool, false>;
  stage(P0{}, 0);
  tile(P0{}, std::integral_constant<bool, true>{}, 0);
  int kt = 1;
  for (; kt + 1 < n_kt; kt += 2) {
    tile(P1{}, F{}, kt);
    tile(P0{}, F{}, kt + 1);
  }
  if (kt < n_kt) tile(P1{}, F{}, kt);

  // normalise and stage O (q rows x 64 hd, bf16) through LDS for coalesced stores
  __syncthreads();
  bf16_t* os = reinterpret_cast<bf16_t*>(smem) + wave * 32 * HD;  // 4 KB per wave
  const float inv_l = 1.0f / l_run;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = db * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      os[(lane & 31) * HD + d] = f2bf(o[db][r] * inv_l);
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int chunk = i * 64 + lane;
    const int qr = chunk >> 3, cc = chunk & 7;
    const int q = qt * AQ + wave * 32 + qr;
    if (q < T) {
      const uint4 v = *reinterpret_cast<const uint4*>(os + qr * HD + cc * 8);
      *reinterpret_cast<uint4*>(out + ((int64_t)b * T + q) * (H * HD) + h * HD + cc * 8) = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// encoder attention, f32 (parity mode): 4 waves = 4 queries share K/V tiles in LDS
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_fwd_f32(const float* __restrict__ qkv, int B, int H, int T,
                                                   float* __restrict__ out) {
  __shared__ float ks[64][HD + 1];
  __shared__ float vs[64][HD + 1];
  __shared__ float qs[4][HD];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_qb = (T + 3) / 4;
  const int bh = blockIdx.x / n_qb, qb = blockIdx.x - bh * n_qb;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int64_t head_elems = (int64_t)T * HD;
  const float* Q = qkv + ((int64_t)(0 * B + b) * H + h) * head_elems;
  const float* K = qkv + ((int64_t)(1 * B + b) * H + h) * head_elems;
  const float* V = qkv + ((int64_t)(2 * B + b) * H + h) * head_elems;
  const int q = qb * 4 + wave;
  qs[wave][lane] = Q[(int64_t)min(q, T - 1) * HD + lane];
  float m = -INFINITY, l = 0.f, acc = 0.f;
  for (int k0 = 0; k0 < T; k0 += 64) {
    __syncthreads();
    for (int i = tid; i < 64 * HD; i += 256) {
      const int r = i >> 6, c = i & 63;
      const int key = min(k0 + r, T - 1);
      ks[r][c] = K[(int64_t)key * HD + c];
      vs[r][c] = V[(int64_t)key * HD + c];
    }
    __syncthreads();
    float s = 0.f;
#pragma unroll 16
    for (int c = 0; c < HD; ++c) s = fmaf(qs[wave][c], ks[lane][c], s);
    if (k0 + lane >= T) s = -INFINITY;
    const float mt = wave_max(s);
    const float mn = fmaxf(m, mt);
    const float alpha = expf(m - mn);
    const float p = expf(s - mn);
    l = l * alpha + wave_sum(p);
    acc *= alpha;
    for (int j = 0; j < 64; ++j) acc = fmaf(__shfl(p, j, 64), vs[j][lane], acc);
    m = mn;
  }
  if (q < T) out[((int64_t)b * T + q) * (H * HD) + h * HD + lane] = acc / l;
}

// ------------------------------------------------------------------------------------------------
// decoder attention helpers: 8 lanes per 64-wide key/value row (16-B loads, 1-KB wave accesses)
// ------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void load8(const T* p, float v[8]);
template <>
__device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float v[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float v[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <typename T>
__device__ __forceinline__ void copy8(T* dst, const T* src) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
  } else {
    reinterpret_cast<float4*>(dst)[0] = reinterpret_cast<const float4*>(src)[0];
    reinterpret_cast<float4*>(dst)[1] = reinterpret_cast<const float4*>(src)[1];
  }
}

// Softmax-weighted sum over keys [k0, k1) for one query (block of 256 threads = 32 key slots x 8 lanes).
// kp(k)/vp(k) give the row pointers.  Returns (via LDS) m, l and o[64] (unnormalised) to thread 0..63.
template <typename T, typename KP, typename VP>
__device__ __forceinline__ void attend_rows(const float qv[8], int k0, int k1, KP kp, VP vp, float* sc,
                                            float (*red)[65], float* stat, float& m_out, float& l_out,
                                            float& o_out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane & 7, kslot = wave * 8 + (lane >> 3);
  float mx = -INFINITY;
  // 4 rows per lane group in flight (addresses clamped, results masked: loads stay unconditional)
  for (int kb = k0 + kslot; kb < k1; kb += 128) {
    float kv[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j) load8<T>(kp(min(kb + 32 * j, k1 - 1)) + sub * 8, kv[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s = fmaf(qv[i], kv[j][i], s);
      s = kw_sum8(s);
      const int k = kb + 32 * j;
      if (k < k1) {
        if (sub == 0) sc[k - k0] = s;
        mx = fmaxf(mx, s);
      }
    }
  }
  mx = wave_max(mx);
  if (lane == 0) stat[wave] = mx;
  __syncthreads();
  const float m = fmaxf(fmaxf(stat[0], stat[1]), fmaxf(stat[2], stat[3]));
  float sum = 0.f;
  for (int k = tid; k < k1 - k0; k += 256) {
    const float e = expf(sc[k] - m);
    sc[k] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) stat[4 + wave] = sum;
  __syncthreads();
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int kb = k0 + kslot; kb < k1; kb += 128) {
    float vv[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j) load8<T>(vp(min(kb + 32 * j, k1 - 1)) + sub * 8, vv[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kb + 32 * j;
      const float pk = k < k1 ? sc[k - k0] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(pk, k < k1 ? vv[j][i] : 0.f, acc[i]);  // (stale masked rows)
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[kslot][sub * 8 + i] = acc[i];
  __syncthreads();
  m_out = m;
  l_out = (stat[4] + stat[5]) + (stat[6] + stat[7]);
  float o = 0.f;
  if (tid < HD)
    for (int s2 = 0; s2 < 32; ++s2) o += red[s2][tid];
  o_out = o;
}

// ------------------------------------------------------------------------------------------------
// Single-query attention over one chunk of <= 256 keys, every K and V load in flight at once
// (256 threads = 32 key slots x 8 lanes; lane (slot, sub) holds 16 B of rows slot, slot+32, ...).
// Returns the chunk's (m, l) to every thread and the unnormalised o[tid] to threads 0..63.
// ------------------------------------------------------------------------------------------------
template <typename T, typename KP, typename VP>
__device__ __forceinline__ void attend_chunk(const float qv[8], int k0, int k1, KP kp, VP vp, float (*red)[64],
                                             float* stat, float& m_out, float& l_out, float& o_out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane & 7, slot = wave * 8 + (lane >> 3);
  Row8<T> kr[8], vr[8];
  // key groups j past the chunk (k0 + 32j >= k1: workgroup-uniform, e.g. the short self-attention chunks of
  // early decode steps) load nothing, and every use of their registers sits behind the same uniform test
  // (no zero fill: a phi of loaded and zeroed registers made the compiler copy a pending load register and
  // wait vmcnt(0) after the second row load).  kp(k, j) / vp(k, j) must not load either: an address that
  // waits on a load costs a vmcnt(0) per row.  Skipped groups contributed p = 0 before: same results.
  auto act = [&](int j) { return k0 + 32 * j < k1; };
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (act(j)) kr[j] = ld_row8<T>(kp(min(k0 + slot + 32 * j, k1 - 1), j) + sub * 8);
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (act(j)) vr[j] = ld_row8<T>(vp(min(k0 + slot + 32 * j, k1 - 1), j) + sub * 8);
  if constexpr (sizeof(T) == 2) {
    float ql[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ql[i] = qv[i] * LOG2E;
    u32x4 k4[8], v4[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k4[j] = kr[j].u[0];
      v4[j] = vr[j].u[0];
    }
    int nj = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) nj += act(j) ? 1 : 0;
    float mw, lw, acc[8];
    wave_row_bf16(ql, k4, v4, k0, k1, slot, nj, mw, lw, acc);
    if (lane < 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) red[wave][lane * 8 + i] = acc[i];
    }
    if (lane == 0) {
      stat[wave] = mw;
      stat[4 + wave] = lw;
    }
    __syncthreads();
    merge_waves_bf16(stat, red, tid, m_out, l_out, o_out);
    return;
  }
  float sc[8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = -INFINITY;
    if (act(j)) {
      float kv[8];
      unpack8<T>(kr[j], kv);
      float sj = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) sj = fmaf(qv[i], kv[i], sj);
      sj = kw_sum8(sj);
      sc[j] = (k0 + slot + 32 * j < k1) ? sj : -INFINITY;
      mx = fmaxf(mx, sc[j]);
    }
  }
  mx = wave_max(mx);
  if (lane == 0) stat[wave] = mx;
  __syncthreads();
  const float m = fmaxf(fmaxf(stat[0], stat[1]), fmaxf(stat[2], stat[3]));
  float lsum = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (act(j)) {
      const bool valid = k0 + slot + 32 * j < k1;
      const float pj = valid ? expf(sc[j] - m) : 0.f;
      lsum += pj;
      float vv[8];
      unpack8<T>(vr[j], vv);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(pj, valid ? vv[i] : 0.f, acc[i]);  // (stale masked rows: see wave_values_bf16)
    }
  }
  // lanes of one wave with equal sub hold the same dims: reduce over lane bits 3..5
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] = kw_sum_hi(acc[i]);
  }
  lsum = wave_sum(lsum) * 0.125f;  // every row's p was counted by its 8 lanes (exact: power of two)
  if (lane < 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wave][lane * 8 + i] = acc[i];
  }
  if (lane == 0) stat[4 + wave] = lsum;
  __syncthreads();
  m_out = m;
  l_out = (stat[4] + stat[5]) + (stat[6] + stat[7]);
  o_out = tid < HD ? (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]) : 0.f;
}

// Combine of per-chunk partials (m, l, o[64]) published write-through by each chunk's workgroup; the
// last arriver (arrival counter) merges them in chunk order and writes the normalised output row.
template <typename T>
__device__ __forceinline__ void publish_and_combine(float* part, int* cnt, int ns, int split, float m, float l, float o,
                                                    T* out_row, int* last_flag) {
  const int tid = threadIdx.x;
  float* w = part + (int64_t)split * (HD + 2);
  if (tid < HD) __hip_atomic_store(w + 2 + tid, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid == 0) {
    __hip_atomic_store(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w + 1, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last_flag = prev == ns - 1;
    if (prev == ns - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!*last_flag || tid >= HD) return;
  constexpr int NSMAX = 8;
  float ms[NSMAX], ls[NSMAX], os[NSMAX];
#pragma unroll
  for (int q = 0; q < NSMAX; ++q) {
    if (q < ns) {
      ms[q] = __hip_atomic_load(part + q * (HD + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ls[q] = __hip_atomic_load(part + q * (HD + 2) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      os[q] = __hip_atomic_load(part + q * (HD + 2) + 2 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  float M = -INFINITY;
#pragma unroll
  for (int q = 0; q < NSMAX; ++q)
    if (q < ns) M = fmaxf(M, ms[q]);
  float lt = 0.f, ot = 0.f;
#pragma unroll
  for (int q = 0; q < NSMAX; ++q)
    if (q < ns) {
      const float f = chunk_scale<T>(ms[q] - M);
      lt = fmaf(ls[q], f, lt);
      ot = fmaf(os[q], f, ot);
    }
  TypeIO<T>::st(out_row + tid, ot / lt);
}
// Chunk-partial hand-off of the bf16 one-row cross-attention (cross_attn_dma_kernel, xq_cross_kernel) through
// 8-byte {data, tag} granules (MI355X_MICROARCH price list, handoff-1to1: one sc1 store each, sc1 polls, untorn),
// per WAVE: a non-final chunk's waves each publish their own (m_w, l_w, acc_w[64]) -- no barrier, no store
// drain, no counter -- and leave.  The final chunk (dispatched after the others) folds, wave by wave and in
// chunk order, every chunk's partial of that wave with fold_begin / fold_value, then merges the four waves with
// merge_waves_bf16: exactly what cross_attn_row_kernel's waves compute as they stream, so a row's output is
// bitwise the same whichever kernel the batch size selects.  Granules [ns - 1][4 waves][66]; each is re-armed
// (tag 0) by its single consumer.  A poll that outlasts XG_SPIN_LIMIT rounds (a protocol failure, never
// expected) raises the error word and writes NaN, so the failure is loud.
__device__ __forceinline__ void wave_partials_combine(unsigned long long* gr, int ns, int split, float mw, float lw,
                                                      const float (&acc)[8], float (*red)[64], float* stat,
                                                      bf16_t* out_row, int* err) {
  constexpr int G = HD + 2, NSMAX = 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (lane < 8) {  // the wave's partial of dim d = lane*8 + i, read back by lane d of the same wave (in order)
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wave][lane * 8 + i] = acc[i];
  }
  if (split != ns - 1) {  // one contiguous 512-B granule store per wave (whole lines: no partial write-through)
    unsigned long long* w = gr + ((int64_t)split * 4 + wave) * G;
    put_granule(w + 2 + lane, red[wave][lane]);
    if (lane == 0) {
      put_granule(w, mw);
      put_granule(w + 1, lw);
    }
    return;
  }
  // lane d of wave w: every earlier chunk's (m, l, acc[d]) of wave w in flight at once (indices clamped: the
  // loads are unconditional, one round trip), then one check
  float ms[NSMAX - 1], ls[NSMAX - 1], as[NSMAX - 1];
  bool bad = false;
  for (int it = 0; ns > 1; ++it) {
    unsigned long long x[3 * (NSMAX - 1)];
#pragma unroll
    for (int q = 0; q < NSMAX - 1; ++q) {
      const unsigned long long* gq = gr + ((int64_t)min(q, ns - 2) * 4 + wave) * G;
      x[3 * q] = peek_granule(gq);
      x[3 * q + 1] = peek_granule(gq + 1);
      x[3 * q + 2] = peek_granule(gq + 2 + lane);
    }
    bool ready = true;
#pragma unroll
    for (int i = 0; i < 3 * (NSMAX - 1); ++i) ready = ready && (x[i] >> 32) == 1ull;
    if (ready || it >= XG_SPIN_LIMIT) {
      bad = !ready;
#pragma unroll
      for (int q = 0; q < NSMAX - 1; ++q) {
        ms[q] = ready ? __uint_as_float((uint32_t)x[3 * q]) : __uint_as_float(0x7fc00000u);
        ls[q] = __uint_as_float((uint32_t)x[3 * q + 1]);
        as[q] = __uint_as_float((uint32_t)x[3 * q + 2]);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(KW_POLL_SLEEP);
  }
  float M = -INFINITY, Lr = 0.f, A = 0.f;
#pragma unroll
  for (int q = 0; q < NSMAX; ++q) {
    if (q >= ns) break;
    float f0 = 0.f, f1 = 0.f;
    const bool own = q == ns - 1;
    const float a = own ? red[wave][lane] : as[q < NSMAX - 1 ? q : 0];
    const int mode = own ? fold_begin(mw, lw, M, Lr, f0, f1) : fold_begin(ms[q < NSMAX - 1 ? q : 0],
                                                                          ls[q < NSMAX - 1 ? q : 0], M, Lr, f0, f1);
    A = fold_value(mode, A, a, f0, f1);
  }
  if (bad) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // re-arm for the next launch: every value above was consumed by this lane (data dependence)
#pragma unroll
  for (int q = 0; q < NSMAX - 1; ++q)
    if (q < ns - 1) {
      unsigned long long* gq = gr + ((int64_t)q * 4 + wave) * G;
      __hip_atomic_store(gq + 2 + lane, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) {
        __hip_atomic_store(gq, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gq + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  __syncthreads();  // every wave has read its own red[] row: reuse red / stat for the folded partials
  red[wave][lane] = A;
  if (lane == 0) {
    stat[wave] = M;
    stat[4 + wave] = Lr;
  }
  __syncthreads();
  if (tid < HD) {
    float m, l, o;
    merge_waves_bf16(stat, red, tid, m, l, o);
    TypeIO<bf16_t>::st(out_row + tid, o / l);
  }
}

// ------------------------------------------------------------------------------------------------
// decoder self-attention: append to the static cache, then causal attention (q_len >= 1).
// New keys/values are read from the qkv rows themselves (never read back from the cache in the
// same launch).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void self_attn_step(const T* __restrict__ qkv, int q_len, int H, T* __restrict__ kc,
                                                      T* __restrict__ vc, int t_max, const int32_t* __restrict__ cur_len,
                                                      T* __restrict__ out) {
  __shared__ float sc[512];
  __shared__ float red[32][65];
  __shared__ float stat[8];
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int sub = lane & 7;
  const int L = *cur_len;
  const int d = H * HD;
  const int p0 = L - q_len;
  T* kb = kc + ((int64_t)b * H + h) * t_max * HD;
  T* vb = vc + ((int64_t)b * H + h) * t_max * HD;
  for (int i = tid; i < q_len * 8; i += 256) {
    const int qi = i >> 3, c8 = i & 7;
    const T* row = qkv + ((int64_t)b * q_len + qi) * 3 * d + h * HD + c8 * 8;
    copy8<T>(kb + (int64_t)(p0 + qi) * HD + c8 * 8, row + d);
    copy8<T>(vb + (int64_t)(p0 + qi) * HD + c8 * 8, row + 2 * d);
  }
  auto kp = [&](int k) -> const T* {
    return k < p0 ? kb + (int64_t)k * HD : qkv + ((int64_t)b * q_len + (k - p0)) * 3 * d + d + h * HD;
  };
  auto vp = [&](int k) -> const T* {
    return k < p0 ? vb + (int64_t)k * HD : qkv + ((int64_t)b * q_len + (k - p0)) * 3 * d + 2 * d + h * HD;
  };
  for (int qi = 0; qi < q_len; ++qi) {
    float qv[8];
    load8<T>(qkv + ((int64_t)b * q_len + qi) * 3 * d + h * HD + sub * 8, qv);
    float m, l, o;
    attend_rows<T>(qv, 0, p0 + qi + 1, kp, vp, sc, red, stat, m, l, o);
    if (tid < HD) TypeIO<T>::st(out + ((int64_t)b * q_len + qi) * d + h * HD + tid, o / l);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// decoder cross-attention: split-S partial softmax; the last-arriving split of a (row, head) combines
// (arrival counter, agent-scope release/acquire -- placement independent).
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void cross_attn_kernel(const T* __restrict__ q, int q_len, int H,
                                                         const T* __restrict__ kc, const T* __restrict__ vc, int S,
                                                         int chunk, float* __restrict__ ws, int* __restrict__ cnt,
                                                         T* __restrict__ out) {
  __shared__ float red[4][64];
  __shared__ float stat[8];
  __shared__ int last;
  const int row = blockIdx.x;  // (b*q_len + qi)*H + h
  const int split = blockIdx.y;
  const int ns = gridDim.y;
  const int h = row % H;
  const int bq = row / H;
  const int b = bq / q_len;
  const int sub = threadIdx.x & 7;
  const int k0 = split * chunk;
  const int k1 = min(S, k0 + chunk);
  const T* kb = kc + ((int64_t)b * H + h) * S * HD;
  const T* vb = vc + ((int64_t)b * H + h) * S * HD;
  float qv[8];
  load8<T>(q + (int64_t)bq * H * HD + h * HD + sub * 8, qv);
  float m, l, o;
  attend_chunk<T>(qv, k0, k1, [&](int k, int) { return kb + (int64_t)k * HD; },
                  [&](int k, int) { return vb + (int64_t)k * HD; }, red, stat, m, l, o);
  T* orow = out + (int64_t)bq * H * HD + h * HD;
  if (ns == 1) {
    if (threadIdx.x < HD) TypeIO<T>::st(orow + threadIdx.x, o / l);
    return;
  }
  publish_and_combine<T>(ws + (int64_t)row * ns * (HD + 2), cnt + row, ns, split, m, l, o, orow, &last);
}

// Cross-attention, bf16, one query row per (row, chunk) workgroup -- as cross_attn_kernel, but the chunk's K
// rows arrive by LDS-DMA (global_load_lds_dwordx4, non-temporal) and V by register loads (r02: 44.4-44.6 us vs
// 45.4-45.6 for register loads only, 50.3 with V by LDS-DMA too at 2 workgroups per CU).  Wave w's DMA
// instruction j moves keys k0 + 32 j + 8 w + (0..7) (1 KB, lane = (key, 16-B piece)) to LDS piece 4 j + w and
// each lane reads back exactly its own 16 B, so the arithmetic is wave_row_bf16's (bitwise the rows of
// cross_attn_kernel / cross_attn_multi_kernel).  r03 (tools/lab/xa_lab.hip, large-v3 B = 32 over 32 distinct
// layers): the same grid only STREAMING its bytes reaches 38-40 us (6.1-6.5 TB/s); the softmax work after
// the loads land costs the rest -- log2-unit scores with per-wave references (no mid-chunk barrier) and DPP
// sums take ~2 us of it, the granule combine (no store drain / counter round trips) another ~1 us.
#ifndef KW_XA_DMA
#define KW_XA_DMA 1  // 0: register loads only (cross_attn_kernel)
#endif
constexpr int XA_DMA = KW_XA_DMA;

// a workgroup barrier without __syncthreads()'s fence (which waits vmcnt(0), draining loads still in flight);
// compiler barriers on both sides keep every memory access (LDS reads of DMA'd data) on its side
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void glds16_nt(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 2);
}
__device__ __forceinline__ u32x4 lds_rd16(const char* p) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_u32(p)) : "memory");
  return v;
}

__global__ __launch_bounds__(256) void cross_attn_dma_kernel(const bf16_t* __restrict__ q, int q_len, int H,
                                                             const bf16_t* __restrict__ kc,
                                                             const bf16_t* __restrict__ vc, int S, int chunk,
                                                             unsigned long long* __restrict__ gran, int* __restrict__ err,
                                                             bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char kv[32 * 1024];
  __shared__ float red[4][64];
  __shared__ float stat[8];
  const int row = blockIdx.x, split = blockIdx.y, ns = gridDim.y;
  const int h = row % H, bq = row / H, b = bq / q_len;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);
  const bf16_t* kb = kc + ((int64_t)b * H + h) * S * HD;
  const bf16_t* vb = vc + ((int64_t)b * H + h) * S * HD;
  // the query first (inline asm: hipcc would otherwise drain every LDS-DMA in flight before its use)
  u32x4 qraw;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qraw) : "v"(q + (int64_t)bq * H * HD + h * HD + sub * 8) : "memory");
  // every group j is issued (clamped keys: the host guarantees k1 - k0 > 224, so group 7 has valid keys)
#pragma unroll
  for (int j = 0; j < 8; ++j) glds16_nt(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8, kv + (4 * j + wave) * 1024);
  u32x4 vr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) vr[j] = ld_row8<bf16_t>(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8).u[0];
  asm volatile("s_waitcnt vmcnt(8)" : "+v"(qraw) :: "memory");  // q and this wave's K pieces landed (V may fly)
  float ql[8];
  {
    Row8<bf16_t> qr;
    qr.u[0] = qraw;
    unpack8<bf16_t>(qr, ql);
#pragma unroll
    for (int i = 0; i < 8; ++i) ql[i] *= LOG2E;
  }
  // no barrier: each lane reads back only the 16 B its own DMA wrote, complete at the wave's vmcnt
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  u32x4 kr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) kr[j] = lds_rd16(kv + (4 * j + wave) * 1024 + lane * 16);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kr[0]), "+v"(kr[1]), "+v"(kr[2]), "+v"(kr[3]), "+v"(kr[4]), "+v"(kr[5]),
               "+v"(kr[6]), "+v"(kr[7]));
  float mw, lw, acc[8];
  wave_row_bf16(ql, kr, vr, k0, k1, slot, 8, mw, lw, acc);
  wave_partials_combine(gran + (int64_t)row * ns * 4 * (HD + 2), ns, split, mw, lw, acc, red, stat,
                        out + (int64_t)bq * H * HD + h * HD, err);
}

// ------------------------------------------------------------------------------------------------
// The cross-attention block's query projection and attention step in ONE launch (bf16 engine, q_len 1):
// the LayerNorm-fused q projection (TF/models/whisper/modeling_whisper.py:483 encoder_attn_layer_norm,
// :309 q * head_dim^-0.5) and cross_attn_dma_kernel's attention over the item's encoder K/V (:323-356) --
// what kw_dec_linear(xq) followed by kw_cross_attn_step computes in two launches, bit for bit.
//
//  * workgroups [0, n_lin): the query projection, 16 columns each -- dec_linear's arithmetic on 4 waves
//    (decproj.h: its 8 waves as virtual waves, reduced in the same order), published as 8-byte
//    {bf16 x 2, tag} granules [M][d/2];
//  * workgroups [n_lin, n_lin + M H ns): cross_attn_dma_kernel's (row, chunk) work in its dispatch order
//    (every row's chunk 0 first, the combining last chunk last).  The query's 4 granules per lane are loaded
//    BEFORE the chunk's K / V stream is issued and checked once the K pieces land: by then the projection
//    (a few us; the first wave of chunks needs ~10 us to stream its 64 MB) has published, so the K / V stream
//    does not wait on it.  The row's last chunk re-arms the row's query granules after its combine (every
//    other chunk of the row has read them: their partials, polled by the combine, depend on them).
// The projection workgroups wait for nothing and lead the dispatch order; a chunk waits only for them and for
// earlier chunks of its row (cross_attn_dma_kernel's combine), so every wait is on work dispatched before it
// -- resident or finished, whatever else shares the GPU (no co-residency assumption).
// Polls are bounded: a timeout raises the error word and the row's output is NaN.
struct XQP {
  const bf16_t* x;
  int64_t ldx;
  float ln_eps;
  const float* ln_colsum;
  const bf16x8* W;
  const float* bias;
  float scale;
  int M, d, H, n_lin, S, chunk, ns;
  const bf16_t* kc;
  const bf16_t* vc;
  unsigned long long* qg;    // [M][d/2] query granules
  unsigned long long* gran;  // cross_attn_dma_kernel's chunk-partial granules
  int* err;
  bf16_t* out;
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void xq_cross_kernel(XQP p) {
  __shared__ __attribute__((aligned(16))) char kv[32 * 1024];  // K pieces (chunks) / reduction scratch (projection)
  __shared__ float red[4][64];
  __shared__ float stat[8];
  if ((int)blockIdx.x < p.n_lin) {
    proj_publish_granules<false>(ProjArgs{p.x, p.ldx, p.M, p.d, p.d, p.ln_eps, p.ln_colsum, p.W, p.bias, p.scale, p.d, p.err + 1},
                                 blockIdx.x, kv, p.qg);
    return;
  }
  const int rows = p.M * p.H;
  const int r = blockIdx.x - p.n_lin;
  const int row = r % rows, split = r / rows, ns = p.ns;
  const int h = row % p.H, b = row / p.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const int k0 = split * p.chunk, k1 = min(p.S, k0 + p.chunk);
  const bf16_t* kb = p.kc + ((int64_t)b * p.H + h) * p.S * HD;
  const bf16_t* vb = p.vc + ((int64_t)b * p.H + h) * p.S * HD;
  unsigned long long* qg = p.qg + (int64_t)b * (p.d / 2) + h * 32;
  // the query's granules first, then every K piece (LDS-DMA) and V row (inline asm for the query loads: hipcc
  // would otherwise drain the LDS-DMA in flight before their use)
  unsigned long long g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(g[i]) : "v"(qg + sub * 4 + i) : "memory");
#pragma unroll
  for (int j = 0; j < 8; ++j) glds16_nt(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8, kv + (4 * j + wave) * 1024);
  u32x4 vr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) vr[j] = ld_row8<bf16_t>(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8).u[0];
  asm volatile("s_waitcnt vmcnt(8)" : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]) :: "memory");  // q + K landed
  bool ok = ((g[0] & g[1] & g[2] & g[3]) >> 32) == 1ull;
  for (int it = 0; __builtin_amdgcn_ballot_w64(!ok) != 0; ++it) {  // the projection not yet published: poll
    if (it >= XG_SPIN_LIMIT) {
      if (!ok) {
        __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = 0x7fc07fc0ull | (1ull << 32);  // bf16 NaN pairs: the row fails loudly
        ok = true;
      }
      continue;
    }
    __builtin_amdgcn_s_sleep(KW_POLL_SLEEP);
#pragma unroll
    for (int i = 0; i < 4; ++i) g[i] = peek_granule(qg + sub * 4 + i);
    ok = ((g[0] & g[1] & g[2] & g[3]) >> 32) == 1ull;
  }
  float ql[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t wq = (uint32_t)g[i];
    ql[2 * i] = __uint_as_float(wq << 16) * LOG2E;
    ql[2 * i + 1] = __uint_as_float(wq & 0xffff0000u) * LOG2E;
  }
  // no barrier: each lane reads back only the 16 B its own DMA wrote, complete at the wave's vmcnt
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  u32x4 kr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) kr[j] = lds_rd16(kv + (4 * j + wave) * 1024 + lane * 16);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kr[0]), "+v"(kr[1]), "+v"(kr[2]), "+v"(kr[3]), "+v"(kr[4]), "+v"(kr[5]),
               "+v"(kr[6]), "+v"(kr[7]));
  float mw, lw, acc[8];
  wave_row_bf16(ql, kr, vr, k0, k1, slot, 8, mw, lw, acc);
  wave_partials_combine(p.gran + (int64_t)row * ns * 4 * (HD + 2), ns, split, mw, lw, acc, red, stat,
                        p.out + (int64_t)b * p.d + h * HD, p.err);
  if (split == ns - 1 && tid < 32)  // re-arm the row's query for the next launch (every chunk has read it)
    __hip_atomic_store(qg + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// Cross-attention, bf16, q_len 1, ONE workgroup per (row, head) pair looping over the pair's chunks with the
// next chunk's K / V in flight while the current one is computed -- used when every pair fits on the device
// at once (large-v3 B = 32: 640 workgroups, 3 per CU).  The chunk-per-workgroup grid (cross_attn_dma_kernel)
// streams in rounds: every workgroup of a round lands its last byte at about the same time, then computes
// while the memory system idles (tools/lab/xa_lab.hip: the same grid only streaming is 38-40 us, with the
// softmax 44-46).  Here each wave keeps its own running softmax over the pair's chunks (log2-unit scores,
// wave_row_bf16, merged online with exp2 rescales); the four waves merge once at the end -- no chunk
// partials, no combine, no workspace.  With QG the query comes from xq_cross's granules (projection
// workgroups [0, n_lin) first, as xq_cross_kernel) and the pair re-arms them after use.
struct CRP {
  const bf16_t* q;           // [rows][64] (row stride d) when !QG
  unsigned long long* qg;    // [M][d/2] query granules when QG
  const bf16_t* kc;
  const bf16_t* vc;
  int H, d, S, chunk, ns, n_lin;
  int* err;
  bf16_t* out;
  ProjArgs proj;  // QG: the query projection
};

// a chunk's 16-B pieces of the pair's K or V rows (lane: row k0 + slot + 32 j, bytes voff = (slot * 64 + sub * 8) * 2
// of it) through a buffer resource over the pair's S rows: rows past S read as 0 (masked like every row past the
// chunk end), so no per-piece clamp or 64-bit address arithmetic -- one add per piece
__device__ __forceinline__ void row_issue(__amdgpu_buffer_rsrc_t rs, int k0, uint32_t voff, u32x4 (&r)[8]) {
  __builtin_amdgcn_sched_barrier(0);  // issue exactly here: the schedule is the point (the compiler would sink these
#pragma unroll                        // loads below the next chunk's arithmetic and wait on them there)
  for (int j = 0; j < 8; ++j)
    r[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + (uint32_t)((k0 + 32 * j) * HD * 2), 0, 2));
  __builtin_amdgcn_sched_barrier(0);
}

// one chunk of the pair: its scores from K (then the caller's next V load goes out, the K registers being dead),
// its values from V, merged into the wave's running (M, Lr, A).  Every chunk holds more than 224 keys (the host's
// row_kernel_fits), so only key group j = 7 can fall past the chunk end.
constexpr int ROW_JV = 7;
__device__ __forceinline__ void row_fold(float mw, const float (&sc)[8], const u32x4 (&vr)[8], int k0, int k1, int slot,
                                         float& M, float& Lr, float (&A)[8]) {
  float lw, acc[8], f0 = 0.f, f1 = 0.f;
  wave_values_bf16<32, ROW_JV>(sc, mw, vr, k0, k1, slot, 8, lw, acc);
  // m_w and l_w come out of full-wave butterflies (commutative adds / maxima: every lane holds the same bits), so
  // lane 0's copy IS the value: read as scalars, (M, Lr) and the fold mode are scalar and the fold is a scalar
  // branch, not eight exec-masked ones per chunk
  const float mu = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, mw)));
  const float lu = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, lw)));
  const int mode = fold_begin(mu, lu, M, Lr, f0, f1);
#pragma unroll
  for (int i = 0; i < 8; ++i) A[i] = fold_value(mode, A[i], acc[i], f0, f1);
}

template <bool QG, int NS>  // NS chunks per pair (6 for Whisper's 1500 frames): a static schedule, static load counts
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void cross_attn_row_kernel(CRP p) {
  __shared__ __attribute__((aligned(16))) char scratch[QG ? PROJ_SCRATCH : 16];
  __shared__ float red[4][64];
  __shared__ float stat[8];
  if constexpr (QG) {
    if ((int)blockIdx.x < p.n_lin) {
      proj_publish_granules<true>(p.proj, blockIdx.x, scratch, p.qg);
      return;
    }
  }
  const int row = blockIdx.x - (QG ? p.n_lin : 0);
  const int h = row % p.H, b = row / p.H;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const bf16_t* kb = p.kc + ((int64_t)b * p.H + h) * p.S * HD;
  const bf16_t* vb = p.vc + ((int64_t)b * p.H + h) * p.S * HD;
  unsigned long long* qg = QG ? p.qg + (int64_t)b * (p.d / 2) + h * 32 : nullptr;
  // the query's loads first, then the first two chunks' K / V
  unsigned long long g[4];
  u32x4 qraw;
  if constexpr (QG) {
#pragma unroll
    for (int i = 0; i < 4; ++i) g[i] = peek_granule(qg + sub * 4 + i);
  } else {
    qraw = *reinterpret_cast<const u32x4*>(p.q + (int64_t)b * p.d + h * HD + sub * 8);
  }
  constexpr int ns = NS;
  const int chunk = p.chunk, S = p.S;
  const __amdgpu_buffer_rsrc_t rsk = __builtin_amdgcn_make_buffer_rsrc((void*)kb, (short)0, S * HD * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsv = __builtin_amdgcn_make_buffer_rsrc((void*)vb, (short)0, S * HD * 2, 0x00020000);
  const uint32_t voff = (uint32_t)((slot * HD + sub * 8) * 2);
  // three 32-register K / V sets in rotation: chunk c + 1's K goes out before chunk c's scores, its V right
  // after them (into chunk c's dead K registers), chunk c + 2's K after chunk c's values (into its dead V
  // registers) -- one chunk in flight while one is computed, 96 K / V registers live
  u32x4 r0[8], r1[8], r2[8];
  row_issue(rsk, 0, voff, r0);
  row_issue(rsv, 0, voff, r1);
  if (ns > 1) row_issue(rsk, chunk, voff, r2);
  if constexpr (QG) {
    bool ok = ((g[0] & g[1] & g[2] & g[3]) >> 32) == 1ull;
    for (int it = 0; __builtin_amdgcn_ballot_w64(!ok) != 0; ++it) {  // the projection not yet published: poll
      if (it >= XG_SPIN_LIMIT) {
        if (!ok) {
          __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int i = 0; i < 4; ++i) g[i] = 0x7fc07fc0ull | (1ull << 32);  // bf16 NaN pairs: the row fails loudly
          ok = true;
        }
        continue;
      }
      __builtin_amdgcn_s_sleep(KW_POLL_SLEEP);
#pragma unroll
      for (int i = 0; i < 4; ++i) g[i] = peek_granule(qg + sub * 4 + i);
      ok = ((g[0] & g[1] & g[2] & g[3]) >> 32) == 1ull;
    }
    qraw = u32x4{(uint32_t)g[0], (uint32_t)g[1], (uint32_t)g[2], (uint32_t)g[3]};
  }
  float ql[8];
  {
    Row8<bf16_t> qr;
    qr.u[0] = qraw;
    unpack8<bf16_t>(qr, ql);
#pragma unroll
    for (int i = 0; i < 8; ++i) ql[i] *= LOG2E;
  }
  float M = -INFINITY, Lr = 0.f, A[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) A[i] = 0.f;
  // chunk c: K in rk, V in rv (the next chunk's K already in the third set); after the step V(c + 1) is in rk
  // and K(c + 2) in rv
  auto step = [&](const int c, u32x4 (&rk)[8], u32x4 (&rv)[8]) __attribute__((always_inline)) {
    float sc[8];
    const int k0 = c * chunk, k1 = min(S, k0 + chunk);
    const float mw = wave_scores_bf16<32, ROW_JV>(ql, rk, k0, k1, slot, 8, sc);
    if (c + 1 < ns) row_issue(rsv, k1, voff, rk);
    row_fold(mw, sc, rv, k0, k1, slot, M, Lr, A);
    if (c + 2 < ns) row_issue(rsk, k0 + 2 * chunk, voff, rv);
  };
#pragma unroll
  for (int c = 0; c < ns; c += 3) {
    step(c, r0, r1);                      // K(c) r0, V(c) r1 -> V(c+1) r0, K(c+2) r1
    if (c + 1 < ns) step(c + 1, r2, r0);  // K(c+1) r2, V(c+1) r0 -> V(c+2) r2, K(c+3) r0
    if (c + 2 < ns) step(c + 2, r1, r2);  // K(c+2) r1, V(c+2) r2 -> V(c+3) r1, K(c+4) r2
  }
  if (lane < 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wave][lane * 8 + i] = A[i];
  }
  if (lane == 0) {
    stat[wave] = M;
    stat[4 + wave] = Lr;
  }
  __syncthreads();
  float m, l, o;
  merge_waves_bf16(stat, red, tid, m, l, o);
  if (tid < HD) TypeIO<bf16_t>::st(p.out + (int64_t)b * p.d + h * HD + tid, o / l);
  if constexpr (QG) {
    if (tid < 32)  // re-arm the row's query for the next launch (every wave of this, its only reader, has read it)
      __hip_atomic_store(qg + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Cross-attention for several query rows of one item (the prefill's P prompt positions, and the beams of
// an item, which all read the same encoder K/V): QN rows per workgroup share ONE pass over the chunk's
// K/V (the one-row kernel above reads it once per row).  Per row the arithmetic is attend_chunk's,
// operation for operation, and the chunk combine is publish_and_combine's, so results are bitwise those
// of cross_attn_kernel.  Rows: r = b*q_len + qi, grouped QN at a time within an item.
template <typename T, int QN>
__global__ __launch_bounds__(256) void cross_attn_multi_kernel(const T* __restrict__ q, int q_len, int H,
                                                               const T* __restrict__ kc, const T* __restrict__ vc,
                                                               int S, int chunk, float* __restrict__ ws,
                                                               int* __restrict__ cnt, T* __restrict__ out) {
  static_assert(QN % 4 == 0 && QN <= 8, "rows in blocks of 4, at most 8 (the beam limit)");
  static_assert(sizeof(T) == 2, "bf16 rows (wave_row_bf16)");
  __shared__ float red[4][4][64];
  __shared__ float stat[4][8];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ngrp = (q_len + QN - 1) / QN;
  const int h = blockIdx.x % H;
  const int bg = blockIdx.x / H;
  const int b = bg / ngrp, qi0 = (bg - b * ngrp) * QN;
  const int nq = min(QN, q_len - qi0);
  const int split = blockIdx.y, ns = gridDim.y;
  const int sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);
  const T* kb = kc + ((int64_t)b * H + h) * S * HD;
  const T* vb = vc + ((int64_t)b * H + h) * S * HD;
  // every load in flight before any arithmetic: the group's query rows (clamped to its last row: no branch),
  // then the chunk's K and V rows; the scheduling barrier keeps the compiler from sinking the V loads below
  // the first row's scores (which put a vmcnt(0) between the K and V streams and another before each later
  // row's query load)
  Row8<T> qr[QN];
#pragma unroll
  for (int r = 0; r < QN; ++r) {
    const T* qp = q + ((int64_t)(b * q_len + qi0 + min(r, nq - 1))) * H * HD + h * HD + sub * 8;
    qr[r].u[0] = *reinterpret_cast<const u32x4*>(qp);
    if constexpr (sizeof(T) == 4) qr[r].u[1] = *(reinterpret_cast<const u32x4*>(qp) + 1);
  }
  Row8<T> kr[8], vr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) kr[j] = ld_row8<T>(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) vr[j] = ld_row8<T>(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
  __builtin_amdgcn_sched_barrier(0);
  // rows in blocks of 4 (one combine thread per (row, dim) per block): the K/V registers stay live
  // across the blocks, so an item's QN rows cost ONE K/V pass
  constexpr int NB = QN / 4;
  float mrow[NB], lrow[NB], orow_acc[NB];  // this thread's row (block bk, row tid / 64): m, l, o[lane]
  u32x4 k4[8], v4[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k4[j] = kr[j].u[0];
    v4[j] = vr[j].u[0];
  }
#pragma unroll
  for (int r0 = 0; r0 < QN; r0 += 4) {
    if (r0 >= nq) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r0 + r >= nq) break;  // (uniform: rows past the group's last are neither computed nor read)
      float ql[8];
      unpack8<T>(qr[r0 + r], ql);
#pragma unroll
      for (int i = 0; i < 8; ++i) ql[i] *= LOG2E;
      float mw, lw, acc[8];
      wave_row_bf16(ql, k4, v4, k0, k1, slot, 8, mw, lw, acc);
      if (lane < 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) red[r][wave][lane * 8 + i] = acc[i];
      }
      if (lane == 0) {
        stat[r][wave] = mw;
        stat[r][4 + wave] = lw;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r == (tid >> 6)) merge_waves_bf16(stat[r], red[r], lane, mrow[r0 / 4], lrow[r0 / 4], orow_acc[r0 / 4]);
    __syncthreads();  // stat / red are rewritten by the next block
  }
  const int dd = lane;
  bool last_any = false;
  if (ns > 1) {
    // publish every owned (row, dim) partial, then one arrival per row group
#pragma unroll
    for (int bk = 0; bk < NB; ++bk) {
      const int rr = bk * 4 + (tid >> 6);
      if (rr < nq) {
        const int row = (b * q_len + qi0 + rr) * H + h;
        float* w = ws + (int64_t)row * ns * (HD + 2) + (int64_t)split * (HD + 2);
        __hip_atomic_store(w + 2 + dd, orow_acc[bk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dd == 0) {
          __hip_atomic_store(w, mrow[bk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(w + 1, lrow[bk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* c = cnt + (b * q_len + qi0) * H + h;  // one counter per row group
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == ns - 1;
      if (prev == ns - 1) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    last_any = last;
    if (!last_any) return;
  }
#pragma unroll
  for (int bk = 0; bk < NB; ++bk) {
    const int rr = bk * 4 + (tid >> 6);
    if (rr >= nq) continue;
    T* orow = out + (int64_t)(b * q_len + qi0 + rr) * H * HD + h * HD;
    if (ns == 1) {
      TypeIO<T>::st(orow + dd, orow_acc[bk] / lrow[bk]);
      continue;
    }
    const int row = (b * q_len + qi0 + rr) * H + h;
    const float* part = ws + (int64_t)row * ns * (HD + 2);
    constexpr int NSMAX = 8;
    float ms[NSMAX], ls[NSMAX], os[NSMAX];
#pragma unroll
    for (int qq = 0; qq < NSMAX; ++qq) {
      if (qq < ns) {
        ms[qq] = __hip_atomic_load(part + qq * (HD + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ls[qq] = __hip_atomic_load(part + qq * (HD + 2) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        os[qq] = __hip_atomic_load(part + qq * (HD + 2) + 2 + dd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    float M = -INFINITY;
#pragma unroll
    for (int qq = 0; qq < NSMAX; ++qq)
      if (qq < ns) M = fmaxf(M, ms[qq]);
    float lt = 0.f, ot = 0.f;
#pragma unroll
    for (int qq = 0; qq < NSMAX; ++qq)
      if (qq < ns) {
        const float f = chunk_scale<T>(ms[qq] - M);
        lt = fmaf(ls[qq], f, lt);
        ot = fmaf(os[qq], f, ot);
      }
    TypeIO<T>::st(orow + dd, ot / lt);
  }
}

// Cross-attention for up to 32 query rows of one item on the matrix cores (beam rows, the beam
// prefill's P x beams positions): the encoder kernel's scheme -- S^T = K Q^T on v_mfma_f32_32x32x16_bf16,
// O^T = V^T P^T with P^T straight from the accumulators and V^T by ds_read_b64_tr_b16 -- on one 64-key
// tile per wave.  The 4 waves of a workgroup cover one <= 256-key chunk with a common row maximum
// (exchanged through LDS) and sum their (l, O) in wave order; the chunks combine as cross_attn_kernel's
// (write-through partials, the last arriver merges in chunk order).  P enters the matrix cores in bf16
// (the one-row kernel keeps it f32): rows agree with it to bf16 rounding, not bitwise.
#ifndef KW_CROSS_MFMA_MIN_Q
#define KW_CROSS_MFMA_MIN_Q 5  // (lab knob: rows per item from which the MFMA kernel takes over)
#endif
constexpr int XM_LDS = 4 * TILE_BYTES;  // per wave: its K, then V, image (32 KB); reused for the (l, O) merge

__global__ __launch_bounds__(256) void cross_attn_mfma_kernel(const bf16_t* __restrict__ q, int q_len, int H,
                                                              const bf16_t* __restrict__ kc,
                                                              const bf16_t* __restrict__ vc, int S, int chunk,
                                                              float* __restrict__ ws, int* __restrict__ cnt,
                                                              bf16_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char xsm[];
  __shared__ float wmax[4][32], wsum[4][32];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, ql = lane & 31;
  const int ngrp = (q_len + 31) / 32;
  const int h = blockIdx.x % H;
  const int bg = blockIdx.x / H;
  const int b = bg / ngrp, qi0 = (bg - b * ngrp) * 32;
  const int nq = min(32, q_len - qi0);
  const int split = blockIdx.y, ns = gridDim.y;
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);
  const int kt0 = k0 + 64 * wave;  // this wave's tile (keys past k1 are masked)
  const bf16_t* K = kc + ((int64_t)b * H + h) * S * HD;
  const bf16_t* V = vc + ((int64_t)b * H + h) * S * HD;
  // one 8-KB LDS image per wave: K lands there by LDS-DMA; V (loaded at the same time, into registers,
  // 16 B per lane per 8-row group) is written over it once the scores are computed
  char* kb = xsm + wave * TILE_BYTES;
  u32x4 vreg[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) {  // 64 rows x 128 B, XOR-swizzled as the encoder's K / V images
    const int row = 8 * g + (lane >> 3);
    const int key = min(kt0 + row, k1 - 1);
    const int slot = lane & 7;
    glds16(K + (int64_t)key * HD + (slot ^ ((row >> 1) & 7)) * 8, kb + g * 1024);
    vreg[g] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(V + (int64_t)key * HD + slot * 8));
  }
  // Q fragments (B operand of S^T = K Q^T): lane holds Q[row ql][16s + 8hh .. +7]
  bf16x8 qf[4];
  {
    const bf16_t* qr = q + (int64_t)(b * q_len + qi0 + min(ql, nq - 1)) * H * HD + h * HD;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qr + 16 * s + 8 * hh);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x16 st[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) st[i][r] = 0.f;
    const int row = i * 32 + ql;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 2 * s + hh;
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
      st[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st[i], 0, 0, 0);
    }
  }
  // the wave's K image is consumed (its fragment reads completed before the MFMAs): V over it, in the
  // transposed-read swizzle (LDS ops of one wave complete in order)
  char* vb = kb;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const int row = 8 * g + (lane >> 3), slot = lane & 7;
    *reinterpret_cast<u32x4*>(vb + row * 128 + ((slot ^ (((row >> 1) & 1) << 2)) << 4)) = vreg[g];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // S^T layout: lane holds query ql, keys i*32 + (r&3) + 8*(r>>2) + 4*hh
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (key >= k1) st[i][r] = -INFINITY;
      mx = fmaxf(mx, st[i][r]);
    }
  mx = xor32_max(mx);
  if (hh == 0) wmax[wave][ql] = mx;
  __syncthreads();
  const float m = fmaxf(fmaxf(wmax[0][ql], wmax[1][ql]), fmaxf(wmax[2][ql], wmax[3][ql]));
  const float mneg = -m * LOG2E;
  float rs = 0.f;
  bf16x8 pf[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float p = __builtin_amdgcn_exp2f(fmaf(st[i][8 * s + e], LOG2E, mneg));
        rs += p;
        pf[i][s][e] = (__bf16)p;
      }
  rs = xor32_sum(rs);
  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  {
    const int li = lane & 15, qq = li >> 2, pp = li & 3, grp = (lane >> 4) & 1;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int i = n >> 1, s = n & 1;
      v2u32 t[2][2];
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int row = i * 32 + 16 * s + 8 * half + 4 * hh + qq;
          const int ch = db * 4 + 2 * grp + (pp >> 1);
          const int off = row * 128 + ((ch ^ (((row >> 1) & 1) << 2)) << 4) + (pp & 1) * 8;
          asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(t[db][half]) : "v"(lds_u32(vb + off)));
        }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t[0][0]), "+v"(t[0][1]), "+v"(t[1][0]), "+v"(t[1][1]));
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const v4u32 w = {t[db][0][0], t[db][0][1], t[db][1][0], t[db][1][1]};
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[i][s], o[db], 0, 0, 0);
      }
    }
  }
  // merge the waves: l and O^T (dims db*32 + (r&3) + 8*(r>>2) + 4*hh of query ql) summed in wave order
  if (hh == 0) wsum[wave][ql] = rs;
  __syncthreads();  // every wave is past its tile reads: the K/V images become the merge buffer
  float* mo = reinterpret_cast<float*>(xsm);  // [wave][query 32][dim 64]
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) mo[(wave * 32 + ql) * HD + db * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh] = o[db][r];
  __syncthreads();
  // thread (query tq, 8 dims from td): the chunk's (m, l, o) of its row
  const int tq = tid >> 3, td = (tid & 7) * 8;
  const bool mine = tq < nq;
  const float mq = fmaxf(fmaxf(wmax[0][tq], wmax[1][tq]), fmaxf(wmax[2][tq], wmax[3][tq]));
  const float lq = ((wsum[0][tq] + wsum[1][tq]) + wsum[2][tq]) + wsum[3][tq];
  float ov[8];
#pragma unroll
  for (int e = 0; e < 8; ++e)
    ov[e] = ((mo[(0 * 32 + tq) * HD + td + e] + mo[(1 * 32 + tq) * HD + td + e]) + mo[(2 * 32 + tq) * HD + td + e]) +
            mo[(3 * 32 + tq) * HD + td + e];
  const int row = (b * q_len + qi0 + min(tq, nq - 1)) * H + h;
  bf16_t* orow = out + (int64_t)(b * q_len + qi0 + min(tq, nq - 1)) * H * HD + h * HD + td;
  if (ns == 1) {
    if (mine) {
      const float inv = 1.f / lq;
#pragma unroll
      for (int e = 0; e < 8; ++e) orow[e] = f2bf(ov[e] * inv);
    }
    return;
  }
  float* part = ws + (int64_t)row * ns * (HD + 2);
  if (mine) {
    float* w = part + (int64_t)split * (HD + 2);
#pragma unroll
    for (int e = 0; e < 8; ++e) __hip_atomic_store(w + 2 + td + e, ov[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (td == 0) {
      __hip_atomic_store(w, mq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(w + 1, lq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* c = cnt + (b * q_len + qi0) * H + h;  // one counter per row group
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == ns - 1;
    if (prev == ns - 1) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last || !mine) return;
  constexpr int NSMAX = 8;
  // every partial in flight before the first use: unconditional loads at a clamped chunk index (a load under
  // `qq2 < ns` feeding the fma chain waited vmcnt(0) per load), the chunks past ns masked in the arithmetic
  float ms[NSMAX], ls[NSMAX], op[NSMAX][8];
#pragma unroll
  for (int qq2 = 0; qq2 < NSMAX; ++qq2) {
    const float* pq = part + min(qq2, ns - 1) * (HD + 2);
    ms[qq2] = __hip_atomic_load(pq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ls[qq2] = __hip_atomic_load(pq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int e = 0; e < 8; ++e) op[qq2][e] = __hip_atomic_load(pq + 2 + td + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float M = -INFINITY;
#pragma unroll
  for (int qq2 = 0; qq2 < NSMAX; ++qq2)
    if (qq2 < ns) M = fmaxf(M, ms[qq2]);
  float f[NSMAX], lt = 0.f;
#pragma unroll
  for (int qq2 = 0; qq2 < NSMAX; ++qq2) {
    f[qq2] = qq2 < ns ? expf(ms[qq2] - M) : 0.f;
    if (qq2 < ns) lt = fmaf(ls[qq2], f[qq2], lt);
  }
  const float inv = 1.f / lt;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float ot = 0.f;
#pragma unroll
    for (int qq2 = 0; qq2 < NSMAX; ++qq2)
      if (qq2 < ns) ot = fmaf(op[qq2][e], f[qq2], ot);
    orow[e] = f2bf(ot * inv);
  }
}

// decoder self-attention for one new position (q_len == 1): split 0 appends k/v at L-1; each split
// attends over its <= 256-key chunk of [0, L) (the new row read from qkv, never from the cache in the
// same launch); splits beyond L exit; the last arriving split combines.
template <typename T, bool BP>
__global__ __launch_bounds__(256) void self_attn_step1(const T* __restrict__ qkv, int H, T* __restrict__ kc,
                                                       T* __restrict__ vc, int t_max, const int32_t* __restrict__ cur_len,
                                                       const int32_t* __restrict__ bp, int bp_stride,
                                                       float* __restrict__ ws, int* __restrict__ cnt, T* __restrict__ out) {
  __shared__ float red[4][64];
  __shared__ float stat[8];
  __shared__ int last;
  const int bh = blockIdx.x, split = blockIdx.y;
  const int b = bh / H, h = bh - (bh / H) * H;
  const int tid = threadIdx.x, sub = tid & 7;
  const int L = *cur_len;
  const int d = H * HD;
  const int p0 = L - 1;
  const int k0 = split * 256;
  if (k0 >= L) return;
  const int ns = (L + 255) / 256;
  T* kb = kc + ((int64_t)b * H + h) * t_max * HD;
  T* vb = vc + ((int64_t)b * H + h) * t_max * HD;
  const T* row = qkv + (int64_t)b * 3 * d + h * HD;
  if (split == 0 && tid < 8) {
    copy8<T>(kb + (int64_t)p0 * HD + tid * 8, row + d + tid * 8);
    copy8<T>(vb + (int64_t)p0 * HD + tid * 8, row + 2 * d + tid * 8);
  }
  float qv[8];
  load8<T>(row + sub * 8, qv);
  float m, l, o;
  // beam search: position k of this row lives in cache row bp[b][k] (a shared prefix), else in row b.  The
  // cache rows of this thread's 8 key slots (attend_chunk's k = min(k0 + slot + 32 j, k1 - 1)) are resolved
  // before any K/V load, so the 16 row loads issue back to back (a slot-table load inside the address of
  // each row put a vmcnt(0) before every row load, on the greedy path too)
  const int k1 = min(L, k0 + 256);
  const int kslot = (tid >> 6) * 8 + ((tid & 63) >> 3);
  int32_t crow[8];
  if constexpr (BP) {  // (a separate instantiation: a runtime branch joins with a vmcnt(0) before the K loads)
    const int32_t* bpr = bp + (int64_t)b * bp_stride;
#pragma unroll
    for (int j = 0; j < 8; ++j) crow[j] = bpr[min(k0 + kslot + 32 * j, k1 - 1)];  // < L <= t_max <= bp_stride
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) crow[j] = b;
  }
  auto slot = [&](int k, int j) -> int64_t { return ((int64_t)crow[j] * H + h) * t_max * HD + (int64_t)k * HD; };
  attend_chunk<T>(qv, k0, k1,
                  [&](int k, int j) -> const T* { return k < p0 ? kc + slot(k, j) : row + d; },
                  [&](int k, int j) -> const T* { return k < p0 ? vc + slot(k, j) : row + 2 * d; }, red, stat, m, l, o);
  T* orow = out + (int64_t)b * d + h * HD;
  if (ns == 1) {
    if (tid < HD) TypeIO<T>::st(orow + tid, o / l);
    return;
  }
  publish_and_combine<T>(ws + (int64_t)bh * 2 * (HD + 2), cnt + bh, ns, split, m, l, o, orow, &last);
}

int cross_splits(int64_t S) {
  int ns = (int)((S + 255) / 256);  // <= 256 keys per chunk (attend_chunk); <= 8 chunks (combine)
  if (ns < 1) ns = 1;
  return ns;
}

}  // namespace

extern "C" int kw_attention(int dtype, const void* qkv, int64_t B, int64_t H, int64_t T, int64_t hd, void* out,
                            kw_stream_t stream) {
  if (!qkv || !out || B <= 0 || H <= 0 || T <= 0) return kw_set_error_msg(KW_EINVAL, "kw_attention: invalid arguments");
  if (hd != HD) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_attention: head_dim must be 64");
  hipStream_t s = (hipStream_t)stream;
  const bool ql2 = (dtype & KW_ATTN_Q_LOG2) != 0;
  dtype &= ~KW_ATTN_Q_LOG2;
  if (ql2 && dtype != KW_DT_BF16) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_attention: KW_ATTN_Q_LOG2 is bf16 only");
  if (dtype == KW_DT_BF16) {
    const int64_t grid = B * H * ((T + AQ - 1) / AQ);
    if (ql2)
      hipLaunchKernelGGL(attn_fwd_l2, dim3((unsigned)grid), dim3(256), 0, s, (const bf16_t*)qkv, (int)B, (int)H, (int)T,
                         (bf16_t*)out);
    else
      hipLaunchKernelGGL(attn_fwd_bf16, dim3((unsigned)grid), dim3(256), 0, s, (const bf16_t*)qkv, (int)B, (int)H, (int)T,
                         (bf16_t*)out);
  } else if (dtype == KW_DT_F32) {
    const int64_t grid = B * H * ((T + 3) / 4);
    hipLaunchKernelGGL(attn_fwd_f32, dim3((unsigned)grid), dim3(256), 0, s, (const float*)qkv, (int)B, (int)H, (int)T,
                       (float*)out);
  } else {
    return kw_set_error_msg(KW_EUNSUPPORTED, "kw_attention: dtype");
  }
  KW_CHECK_LAUNCH();
  return KW_OK;
}

extern "C" size_t kw_self_attn_workspace(int64_t B, int64_t H, int64_t t_max) {
  (void)t_max;  // t_max <= 512: at most two 256-key chunks per (b, h)
  return (size_t)(B * H) * 2 * (HD + 2) * sizeof(float) + (size_t)(B * H) * sizeof(int);
}

extern "C" int kw_self_attn_step(int dtype, const void* qkv, int64_t B, int64_t q_len, int64_t H, int64_t hd,
                                 void* k_cache, void* v_cache, int64_t t_max, const int32_t* cur_len,
                                 const int32_t* bp, int64_t bp_stride, void* out, void* workspace, size_t ws_bytes,
                                 kw_stream_t stream) {
  if (!qkv || !k_cache || !v_cache || !cur_len || !out || B <= 0 || q_len <= 0 || H <= 0 || t_max <= 0 || t_max > 512)
    return kw_set_error_msg(KW_EINVAL, "kw_self_attn_step: invalid arguments (t_max <= 512)");
  if (hd != HD) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_self_attn_step: head_dim must be 64");
  hipStream_t s = (hipStream_t)stream;
  if (bp && (q_len != 1 || bp_stride < t_max))
    return kw_set_error_msg(KW_EINVAL, "kw_self_attn_step: a slot table needs q_len == 1 and bp_stride >= t_max");
  if (q_len == 1) {
    if (!workspace || ws_bytes < kw_self_attn_workspace(B, H, t_max))
      return kw_set_error_msg(KW_EINVAL, "kw_self_attn_step: needs a zero-filled workspace of kw_self_attn_workspace()");
    float* part = (float*)workspace;
    int* cnt = (int*)((char*)workspace + (size_t)(B * H) * 2 * (HD + 2) * sizeof(float));
    dim3 grid((unsigned)(B * H), (unsigned)((t_max + 255) / 256));
    if (dtype == KW_DT_BF16)
      hipLaunchKernelGGL((bp ? self_attn_step1<bf16_t, true> : self_attn_step1<bf16_t, false>), grid, dim3(256), 0, s,
                         (const bf16_t*)qkv, (int)H, (bf16_t*)k_cache, (bf16_t*)v_cache, (int)t_max, cur_len, bp,
                         (int)bp_stride, part, cnt, (bf16_t*)out);
    else
      hipLaunchKernelGGL((bp ? self_attn_step1<float, true> : self_attn_step1<float, false>), grid, dim3(256), 0, s,
                         (const float*)qkv, (int)H, (float*)k_cache, (float*)v_cache, (int)t_max, cur_len, bp,
                         (int)bp_stride, part, cnt, (float*)out);
  } else if (dtype == KW_DT_BF16) {
    hipLaunchKernelGGL(self_attn_step<bf16_t>, dim3((unsigned)(B * H)), dim3(256), 0, s, (const bf16_t*)qkv, (int)q_len,
                       (int)H, (bf16_t*)k_cache, (bf16_t*)v_cache, (int)t_max, cur_len, (bf16_t*)out);
  } else {
    hipLaunchKernelGGL(self_attn_step<float>, dim3((unsigned)(B * H)), dim3(256), 0, s, (const float*)qkv, (int)q_len,
                       (int)H, (float*)k_cache, (float*)v_cache, (int)t_max, cur_len, (float*)out);
  }
  KW_CHECK_LAUNCH();
  return KW_OK;
}

static size_t cross_partials_bytes(int64_t B, int64_t q_len, int64_t H, int64_t S) {
  return (size_t)(B * q_len * H) * cross_splits(S) * (HD + 2) * sizeof(float);
}

// workspace: f32 partials [rows][ns][HD+2] | arrival counters [rows] (publish_and_combine kernels) | status word,
// fault-injection word (kw_dec_xq_cross's projection),
// padded to 64 B | 8-byte granules [rows][ns][4 waves][HD+2] (cross_attn_dma_kernel, xq_cross_kernel); every region
// zero before first use
static size_t cross_granule_offset(int64_t B, int64_t q_len, int64_t H, int64_t S) {
  const size_t head = cross_partials_bytes(B, q_len, H, S) + (size_t)(B * q_len * H) * sizeof(int) + 2 * sizeof(int);
  return (head + 63) & ~(size_t)63;
}

extern "C" size_t kw_cross_attn_workspace(int64_t B, int64_t q_len, int64_t H, int64_t hd, int64_t S) {
  (void)hd;
  return cross_granule_offset(B, q_len, H, S) + 8 * cross_partials_bytes(B, q_len, H, S);  // granules per wave
}

extern "C" size_t kw_cross_attn_status_offset(int64_t B, int64_t q_len, int64_t H, int64_t hd, int64_t S) {
  (void)hd;
  return cross_partials_bytes(B, q_len, H, S) + (size_t)(B * q_len * H) * sizeof(int);
}

// cross_attn_row_kernel when one round of pair workgroups covers the device -- at least one per CU, all resident
// at once (the occupancy query) -- and the A/B switch KW_CROSS_ROW=0 is not set (read once).
constexpr int ROW_NS = 6;  // cross_attn_row_kernel's chunk count (S = 1500)

template <bool QG>
static bool row_kernel_fits(int64_t rows, int64_t S) {
  const int ns = cross_splits(S);
  const int64_t chunk = (S + ns - 1) / ns;
  if (chunk <= 32 * ROW_JV || S - (int64_t)(ns - 1) * chunk <= 32 * ROW_JV) return false;  // row_fold's key groups
  static int ncu = 0, per_cu = 0, off = -1;
  if (off < 0) {
    const char* e = getenv("KW_CROSS_ROW");
    off = (e && e[0] == '0') ? 1 : 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&cross_attn_row_kernel<QG, ROW_NS>), 256,
                                                     0) != hipSuccess)
      ncu = per_cu = 0;
  }
  return !off && ns == ROW_NS && ncu > 0 && rows >= ncu && rows <= (int64_t)ncu * per_cu;
}

extern "C" int kw_cross_attn_pair_kernel(int64_t rows, int64_t S, int fused) {
  return (fused ? row_kernel_fits<true>(rows, S) : row_kernel_fits<false>(rows, S)) ? 1 : 0;
}

extern "C" int kw_cross_attn_step(int dtype, const void* q, int64_t B, int64_t q_len, int64_t H, int64_t hd,
                                  const void* k, const void* v, int64_t S, void* out, void* workspace, size_t ws_bytes,
                                  kw_stream_t stream) {
  if (!q || !k || !v || !out || !workspace || B <= 0 || q_len <= 0 || H <= 0 || S <= 0)
    return kw_set_error_msg(KW_EINVAL, "kw_cross_attn_step: invalid arguments");
  if (hd != HD) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_cross_attn_step: head_dim must be 64");
  if (ws_bytes < kw_cross_attn_workspace(B, q_len, H, hd, S))
    return kw_set_error_msg(KW_EINVAL, "kw_cross_attn_step: workspace too small");
  if (S > 2048) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_cross_attn_step: S <= 2048 (8 chunks of 256)");
  const int ns = cross_splits(S);
  const int chunk = (int)((S + ns - 1) / ns);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)(B * q_len * H), (unsigned)ns);
  float* part = (float*)workspace;
  int* cnt = (int*)((char*)workspace + cross_partials_bytes(B, q_len, H, S));
  if (dtype == KW_DT_BF16 && q_len > 1 && q_len <= 4) {  // several rows per item (prefill, beams): one K/V pass
    const dim3 gm((unsigned)(B * H), (unsigned)ns);
    hipLaunchKernelGGL((cross_attn_multi_kernel<bf16_t, 4>), gm, dim3(256), 0, s, (const bf16_t*)q, (int)q_len, (int)H,
                       (const bf16_t*)k, (const bf16_t*)v, (int)S, chunk, part, cnt, (bf16_t*)out);
  } else if (dtype == KW_DT_BF16 && q_len >= KW_CROSS_MFMA_MIN_Q) {  // beams: up to 32 rows per pass, MFMA
    static bool attr = false;
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cross_attn_mfma_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, XM_LDS);
      if (e != hipSuccess) return kw_set_error(e);
      attr = true;
    }
    const dim3 gm((unsigned)(B * ((q_len + 31) / 32) * H), (unsigned)ns);
    hipLaunchKernelGGL(cross_attn_mfma_kernel, gm, dim3(256), XM_LDS, s, (const bf16_t*)q, (int)q_len, (int)H,
                       (const bf16_t*)k, (const bf16_t*)v, (int)S, chunk, part, cnt, (bf16_t*)out);
  } else if (dtype == KW_DT_BF16 && q_len > 4) {  // up to 8 rows per K/V pass, groups of 8 beyond
    const dim3 gm((unsigned)(B * ((q_len + 7) / 8) * H), (unsigned)ns);
    hipLaunchKernelGGL((cross_attn_multi_kernel<bf16_t, 8>), gm, dim3(256), 0, s, (const bf16_t*)q, (int)q_len, (int)H,
                       (const bf16_t*)k, (const bf16_t*)v, (int)S, chunk, part, cnt, (bf16_t*)out);
  } else if (dtype == KW_DT_BF16 && q_len == 1 && row_kernel_fits<false>(B * H, S)) {
    CRP p{};
    p.q = (const bf16_t*)q;
    p.kc = (const bf16_t*)k;
    p.vc = (const bf16_t*)v;
    p.H = (int)H, p.d = (int)(H * HD), p.S = (int)S, p.chunk = chunk, p.ns = ns, p.n_lin = 0;
    p.err = cnt + B * q_len * H;
    p.out = (bf16_t*)out;
    hipLaunchKernelGGL((cross_attn_row_kernel<false, ROW_NS>), dim3((unsigned)(B * H)), dim3(256), 0, s, p);
  } else if (dtype == KW_DT_BF16 && XA_DMA && chunk > 224 && chunk <= 256 && S - (int64_t)(ns - 1) * chunk > 224)
    hipLaunchKernelGGL(cross_attn_dma_kernel, grid, dim3(256), 0, s, (const bf16_t*)q, (int)q_len, (int)H,
                       (const bf16_t*)k, (const bf16_t*)v, (int)S, chunk,
                       (unsigned long long*)((char*)workspace + cross_granule_offset(B, q_len, H, S)),
                       cnt + B * q_len * H, (bf16_t*)out);
  else if (dtype == KW_DT_BF16)
    hipLaunchKernelGGL(cross_attn_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)q, (int)q_len, (int)H,
                       (const bf16_t*)k, (const bf16_t*)v, (int)S, chunk, part, cnt, (bf16_t*)out);
  else
    hipLaunchKernelGGL(cross_attn_kernel<float>, grid, dim3(256), 0, s, (const float*)q, (int)q_len, (int)H,
                       (const float*)k, (const float*)v, (int)S, chunk, part, cnt, (float*)out);
  KW_CHECK_LAUNCH();
  return KW_OK;
}

static size_t xq_gran_offset(int64_t M, int64_t H, int64_t S) {
  return (kw_cross_attn_workspace(M, 1, H, HD, S) + 63) & ~(size_t)63;
}

static bool xq_shape_ok(int64_t M, int64_t d, int64_t H, int64_t S) {
  if (!proj_shape_ok(M, d) || H < 1 || d != HD * H || S < 1 || S > 2048) return false;
  const int ns = cross_splits(S);
  const int64_t chunk = (S + ns - 1) / ns;
  return ns >= 1 && chunk > 224 && chunk <= 256 && S - (int64_t)(ns - 1) * chunk > 224;  // cross_attn_dma_kernel's
}

extern "C" size_t kw_dec_xq_cross_workspace(int64_t M, int64_t d, int64_t H, int64_t S) {
  if (M < 1 || d < 2 || H < 1 || S < 1) return 0;
  return xq_gran_offset(M, H, S) + (size_t)M * (size_t)(d / 2) * sizeof(unsigned long long);
}

extern "C" size_t kw_dec_xq_cross_status_offset(int64_t M, int64_t d, int64_t H, int64_t S) {
  (void)d;
  return kw_cross_attn_status_offset(M, 1, H, HD, S);  // status word, then the fault-injection word
}

extern "C" int kw_dec_xq_cross_supported(int64_t M, int64_t d, int64_t H, int64_t S) {
  return xq_shape_ok(M, d, H, S) ? 1 : 0;  // (every wait is on earlier-dispatched work: no residency condition)
}

extern "C" int kw_dec_xq_cross(const kw_dec_xq_cross_args* a, kw_stream_t stream) {
  if (!a || !a->x || !a->W || !a->ln_colsum || !a->k || !a->v || !a->out || !a->workspace)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_xq_cross: null pointer");
  if (!xq_shape_ok(a->M, a->d, a->H, a->S) || a->ldx < a->d || a->ldx % 8 || (uintptr_t)a->x % 16)
    return kw_set_error_msg(KW_EINVAL, "kw_dec_xq_cross: M <= 32 rows, d = 64 H <= 1280, 224 < S / chunks <= 256, "
                                       "ldx % 8 == 0, 16-B aligned x");
  if (a->ws_bytes < kw_dec_xq_cross_workspace(a->M, a->d, a->H, a->S))
    return kw_set_error_msg(KW_EINVAL, "kw_dec_xq_cross: needs a zero-filled workspace of kw_dec_xq_cross_workspace()");
  XQP p;
  p.x = reinterpret_cast<const bf16_t*>(a->x);
  p.ldx = a->ldx;
  p.ln_eps = a->ln_eps;
  p.ln_colsum = a->ln_colsum;
  p.W = reinterpret_cast<const bf16x8*>(a->W);
  p.bias = a->bias;
  p.scale = a->scale;
  p.M = (int)a->M;
  p.d = (int)a->d;
  p.H = (int)a->H;
  p.n_lin = (int)(a->d / 16);
  p.S = (int)a->S;
  p.ns = cross_splits(a->S);
  p.chunk = (int)((a->S + p.ns - 1) / p.ns);
  p.kc = reinterpret_cast<const bf16_t*>(a->k);
  p.vc = reinterpret_cast<const bf16_t*>(a->v);
  char* ws = reinterpret_cast<char*>(a->workspace);
  p.qg = reinterpret_cast<unsigned long long*>(ws + xq_gran_offset(a->M, a->H, a->S));
  p.gran = reinterpret_cast<unsigned long long*>(ws + cross_granule_offset(a->M, 1, a->H, a->S));
  p.err = reinterpret_cast<int*>(ws + cross_partials_bytes(a->M, 1, a->H, a->S)) + a->M * a->H;
  p.out = reinterpret_cast<bf16_t*>(a->out);
  if (row_kernel_fits<true>(a->M * a->H, a->S)) {  // one pair workgroup per (row, head), chunks pipelined
    CRP r{};
    r.qg = p.qg;
    r.kc = p.kc;
    r.vc = p.vc;
    r.H = p.H, r.d = p.d, r.S = p.S, r.chunk = p.chunk, r.ns = p.ns, r.n_lin = p.n_lin;
    r.err = p.err;
    r.out = p.out;
    r.proj = ProjArgs{p.x, p.ldx, p.M, p.d, p.d, p.ln_eps, p.ln_colsum, p.W, p.bias, p.scale, p.d, p.err + 1};
    hipLaunchKernelGGL((cross_attn_row_kernel<true, ROW_NS>), dim3((unsigned)(p.n_lin + a->M * a->H)), dim3(256), 0,
                       (hipStream_t)stream, r);
    KW_CHECK_LAUNCH();
    return KW_OK;
  }
  const int64_t grid = p.n_lin + a->M * a->H * p.ns;
  hipLaunchKernelGGL(xq_cross_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, p);
  KW_CHECK_LAUNCH();
  return KW_OK;
}
