// Decoder cross-attention read straight from the encoder output (a3 cross, TF modeling_whisper.py:
// 284-356 with the cross K/V of :323-335), gfx950.
//
// The reference projects the encoder output e [S][D] of every item into every decoder layer's K and V
// (k = e Wk^T, v = e Wv^T + bv: 2 x 32 layers x S x D values, 7.86 GB at B = 32 in bf16) and streams a
// layer's K and V (245 MB at B = 32) on every decode step.  Both projections are linear, so they move to
// the query and output sides of the attention (per head h, with q_h pre-scaled):
//
//   q_h . k_f = q_h . (Wk_h e_f) = (Wk_h^T q_h) . e_f = u_h . e_f          u_h = Wk_h^T q_h  [D]
//   sum_f p_f v_f = Wv_h (sum_f p_f e_f) + bv_h = Wv_h z_h + bv_h             (sum_f p_f = 1)
//
// u and Wv_h z_h + bv are two small decode linears over packed weights (kw_dec_linear with grouped
// activations, 3.3 MB of weights each at large-v3); this kernel computes, for each item and query,
//   s_f = e_f . u,   p = softmax_f(s),   z = sum_f p_f e_f,
// reading the item's e (S x D bf16 = 3.84 MB at large-v3) ONCE for all H queries of a decoder step, and
// the SAME e for every decoder layer: 123 MB per layer at B = 32 instead of 245 MB of K/V, a working set
// the 256 MB Infinity Cache keeps across the 32 layers of a step (MI355X_MICROARCH "Infinity Cache").
// The cross K/V cache and its 1.0e13-flop projection GEMM disappear from the bf16 engine.
//
// Work split: workgroup = (item, chunk of frames); its NW waves split the D channels (wave w owns
// channels [w*32*KS, (w+1)*32*KS)), so each wave streams only its own channel slice of every 16-frame
// sub-tile (LDS-DMA into a wave-private ring slot, 2 sub-tiles in flight) and needs no other wave's data:
//   * S^T partial over the wave's channels on v_mfma_f32_16x16x32_bf16 (A = e rows, B = u fragments held
//     in registers for the whole launch); the NW partial tiles are summed in wave order through LDS by
//     one wave per 16-query block, which runs the online softmax (running max / sum in f32) and
//     publishes P (bf16) and the rescale factors;
//   * z += P e on v_mfma_f32_16x16x16_bf16 with e's B fragments by ds_read_b64_tr_b16 from the same
//     sub-tile image (16-row x 32-channel 1-KB blocks, chunk XOR (row>>1)&3: conflict-free for both the
//     row reads and the transposed reads);
//   * chunks of one item combine after an item barrier (write-through partials, arrival counter; every
//     chunk's workgroup then merges 1/nch of the channels in chunk order) -- grid <= CUs, so all chunks
//     of an item are resident (and in-order dispatch would keep them so anyway); the spin is bounded.
// Everything is deterministic (fixed-order sums, no float atomics).
#include <math.h>

#include "kw_common.h"

#if KW_XENC_STAMPS
// lab builds only: shader-clock stamps of workgroup 0 (waves 0 and 2), read back by kw_lab_xenc_stamps
__device__ unsigned long long g_xenc_stamps[2][512];
#define XSTAMP(i)                                                                                       \
  do {                                                                                                  \
    if (blockIdx.x == 0 && (wave == 0 || wave == 2) && lane == 0 && (i) < 512)                          \
      g_xenc_stamps[wave >> 1][(i)] = __builtin_amdgcn_s_memtime();                                     \
  } while (0)
#else
#define XSTAMP(i)
#endif

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(2))) unsigned int v2u32;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u32;

constexpr float LOG2E = 1.4426950408889634f;
constexpr int NBUF = 3;      // ring slots per wave (2 sub-tiles in flight while one is consumed)
constexpr int SUB = 16;      // frames per sub-tile
constexpr int HB = 2;        // 16-query blocks per launch
constexpr int QMAX = 16 * HB;
constexpr int NCHMAX = 8;    // chunks per item
constexpr int SPIN_MAX = 1 << 24;
#ifndef KW_XENC_STAMPS
#define KW_XENC_STAMPS 0
#endif
#ifndef KW_XENC_LAB
#define KW_XENC_LAB 0  // lab builds only: 1 = no partial publish / merge loads, 2 = no loop compute, 3 = no loop loads
#endif

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
// LDS accesses of the streaming loop are inline asm: a builtin LDS access after an LDS-DMA would get a
// compiler s_waitcnt vmcnt(0) (it cannot tell the ring slot in use from the ones in flight); the waits
// here are explicit (lgkmcnt before use, counted vmcnt for the ring)
__device__ __forceinline__ bf16x8 ds_rd128(const char* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ f32x4 ds_rd128f(const char* p) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ v2u32 ds_rd64(const char* p) {
  v2u32 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ v2u32 ds_tr64(const char* p) {
  v2u32 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ void ds_wr128f(char* p, f32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
// an MFMA result read by an inline-asm store: the compiler's hazard recognizer does not see the asm's
// operand, so the XDL-write -> LDS-read wait states (11 for an 8-pass MFMA) are inserted here
__device__ __forceinline__ void ds_wr128f_mfma(char* p, f32x4 v) {
  asm volatile("s_nop 7\n\ts_nop 7\n\tds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void ds_wr64(char* p, v2u32 v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void ds_wr32f(char* p, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ float ds_rd32f(const char* p) {
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ void ds_wr16(char* p, uint32_t v) {
  asm volatile("ds_write_b16 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
// write-through (agent-coherent) 16-B global accesses for the chunk partials
__device__ __forceinline__ void st16_sc1(void* p, v4u32 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ v4u32 ld16_sc1(const void* p) {
  v4u32 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// 16-lane row reductions by DPP (xor 1, xor 2, half-row mirror, row mirror): every lane of the row ends
// with the same value (each step combines two operands commutatively)
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// lane ^ 16 / lane ^ 32 exchanges by v_permlane16/32_swap (VALU; no LDS round trip like ds_bpermute): with
// both operands = v, one result is the lane's own value and the other its partner's
__device__ __forceinline__ float xor16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  return fmaxf(v, dppf<0x140>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  return v + dppf<0x140>(v);
}
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() {  // no implicit vmcnt(0) drain (the ring stays in flight)
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <typename T>
__device__ __forceinline__ void tie(T& v) {  // v is used only after the preceding explicit wait
  asm volatile("" : "+v"(v));
}

struct XaP {
  const bf16_t* enc;  // [B][S][D]
  int S, D, H;
  const bf16_t* u;    // [B*q_len][H][D]: query j = r*H + h of this launch's row qi0 + r
  bf16_t* z;          // [B*q_len][H][D]
  int q_len, qi0, Q;  // Q = rows * H queries per item in this launch (<= QMAX)
  int nch, nst;       // chunks per item, 16-frame sub-tiles per item
  float* ml;          // [B*nch][QMAX][2] chunk (max, sum)
  bf16_t* zp;         // [B*nch][QMAX][D] chunk partial z (unnormalised, bf16: half the merge traffic)
  int* cnt;           // [B] arrivals   (zero before, left zero)
  int* dep;           // [B] departures (zero before, left zero)
  int* err;           // [1] set when an item barrier timed out
  int wts_off;        // LDS byte offset of the merge weights (after the partial-transpose image)
};

template <int NW, int KS>
__global__ __launch_bounds__(NW * 64) void xattn_enc_kernel(XaP p) {
  constexpr int CPW = 32 * KS;              // channels per wave (z phase)
  constexpr int WREG = KS * 1024;           // one wave's part of a ring slot
  constexpr int SLOT = NW * WREG;
  constexpr int SB = NW * KS / 2;           // 32-channel blocks of a score wave (half the channels)
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* ring = lds;                                        // [NBUF][NW][KS][1 KB]
  char* red = lds + NBUF * SLOT;                           // [HB][64 lanes] f32x4: second-half partial scores
  char* pimg = red + HB * 64 * 16;                         // [QMAX][16 frames] bf16 (32-B rows): P
  char* alph = pimg + QMAX * 32;                           // [QMAX] f32 rescale factors, then [HB] int flags
  float* wts = reinterpret_cast<float*>(lds + p.wts_off);  // [NCHMAX][QMAX] combine weights

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x / p.nch, c = blockIdx.x - (blockIdx.x / p.nch) * p.nch;
  const int st0 = (p.nst * c) / p.nch, st1 = (p.nst * (c + 1)) / p.nch, nt = st1 - st0;
  const int fend = min(p.S, st1 * SUB);
  const int D = p.D, Q = p.Q;
  const bf16_t* encb = p.enc + (int64_t)b * p.S * D;
  const int ch0 = wave * CPW;
  const int64_t qrow0 = ((int64_t)b * p.q_len + p.qi0) * p.H;  // first query's row in u / z
  // score waves: wave w < 2 HB owns query block hb = w % HB over channel half w / HB
  const bool swave = wave < 2 * HB;
  const int shb = wave % HB, shalf = wave / HB;

  // sub-tile t of this chunk -> ring slot t % NBUF, this wave's channels: KS 1-KB LDS-DMA pieces, piece s =
  // 16 frames x 32 channels, lane i -> frame i>>2, 16-B chunk (i&3) ^ ((frame>>1)&3) of the block
  auto issue = [&](int t) {
    char* dst = ring + (t % NBUF) * SLOT + wave * WREG;
    const int row = lane >> 2, cc = (lane & 3) ^ ((row >> 1) & 3);
    const bf16_t* src = encb + (int64_t)min((st0 + t) * SUB + row, p.S - 1) * D + ch0 + cc * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (KW_XENC_LAB != 3) glds16(src + 32 * s, dst + s * 1024);
    }
  };

  // z accumulators on v_mfma_f32_32x32x16_bf16: block k = channels ch0 + 32k; lane holds channel l&31,
  // queries (r&3) + 8(r>>2) + 4(l>>5)
  f32x16 zacc[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) zacc[k][r] = 0.f;
  // online softmax state (score waves of the first half): query fr + 16 shb, log2 domain, replicated in the
  // query's 4 lanes; the reference max m_ref moves only when a sub-tile's max exceeds it by RESCALE_LOG2
  // (rescaling z is then rare); p = exp2(s - m_ref) <= 2^RESCALE_LOG2
  constexpr float RESCALE_LOG2 = 8.f;
  float m_ref = -INFINITY, l_run = 0.f;

  XSTAMP(0);
  issue(0);
  // u fragments of a score wave (B operand of S = e_rows . u): lane holds u[query 16 shb + (l&15)][32 sb + 8(l>>4) ..]
  // for its half's blocks sb (loaded behind sub-tile 0; the compiler's wait for them drains it too, so the loop's
  // counted vmcnt waits only ever see ring pieces)
  bf16x8 uf[SB];
  {
    const int j = 16 * shb + (lane & 15);
#pragma unroll
    for (int s = 0; s < SB; ++s) {
      if (swave && j < Q) {
        uf[s] = *reinterpret_cast<const bf16x8*>(p.u + (qrow0 + j) * D + 32 * (shalf * SB + s) + 8 * (lane >> 4));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) uf[s][e] = (__bf16)0.0f;
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SB; ++s) tie(uf[s]);
  if (nt > 1) issue(1);  // (behind the compiler's wait for u and sub-tile 0: the loop starts on sub-tile 0 alone)
  const int fr = lane & 15, fg = lane >> 4;  // fragment row / 16-B group
  XSTAMP(1);
  for (int t = 0; t < nt; ++t) {
    if (t + 2 < nt) {
      issue(t + 2);  // into slot (t-1) % NBUF: every wave's reads of it completed before barrier C of step t-1
      vmwait<2 * KS>();
    } else if (t + 1 < nt) {
      vmwait<KS>();
    } else {
      vmwait<0>();
    }
    const char* sl = ring + (t % NBUF) * SLOT;
    XSTAMP(8 + 8 * t);
    raw_barrier();  // A: every wave's pieces of sub-tile t have landed
    if (KW_XENC_LAB == 2) continue;
    // 1. score waves: S[frame 4fg + i][query fr + 16 shb] over their channel half (C layout = the z MFMA's
    //    A-operand layout of P: query on the lane, 4 frames in the registers)
    f32x4 sacc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (swave) {
      auto rd = [&](int s0, bf16x8 (&a)[KS]) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int blk = shalf * SB + s0 + s;  // global 32-channel block -> owning wave's region
          a[s] = ds_rd128(sl + (blk / KS) * WREG + (blk % KS) * 1024 + fr * 64 + ((fg ^ ((fr >> 1) & 3)) << 4));
        }
      };
      bf16x8 a0[KS], a1[KS];
      rd(0, a0);
#pragma unroll
      for (int s0 = 0; s0 < SB; s0 += 2 * KS) {  // reads of the next KS blocks in flight beside the MFMAs
        if (s0 + KS < SB) rd(s0 + KS, a1);
        if (s0 + KS < SB) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(KS) : "memory");
        else lgkm0();
#pragma unroll
        for (int s = 0; s < KS; ++s) tie(a0[s]);
#pragma unroll
        for (int s = 0; s < KS; ++s) sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[s], uf[s0 + s], sacc, 0, 0, 0);
        if (s0 + KS >= SB) break;
        if (s0 + 2 * KS < SB) rd(s0 + 2 * KS, a0);
        if (s0 + 2 * KS < SB) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(KS) : "memory");
        else lgkm0();
#pragma unroll
        for (int s = 0; s < KS; ++s) tie(a1[s]);
#pragma unroll
        for (int s = 0; s < KS; ++s) sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[s], uf[s0 + KS + s], sacc, 0, 0, 0);
      }
      if (shalf == 1) ds_wr128f_mfma(red + (shb * 64 + lane) * 16, sacc);
      lgkm0();
    }
    XSTAMP(9 + 8 * t);
    raw_barrier();  // B: second-half partials published
    XSTAMP(10 + 8 * t);
    // 2. first-half score waves: full scores (halves summed in order), online softmax, P and the rescale factors
    if (swave && shalf == 0) {
      f32x4 other = ds_rd128f(red + (shb * 64 + lane) * 16);
      lgkm0();
      tie(other);
      // (the MFMA result sacc is read by VALU here: the compiler inserts the wait states)
      f32x4 sc = sacc + other;
      const int f0 = (st0 + t) * SUB + 4 * fg;
      float mt = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sc[i] = f0 + i < fend ? sc[i] * LOG2E : -INFINITY;
        mt = fmaxf(mt, sc[i]);
      }
      mt = xor32_max(xor16_max(mt));
      const bool bump = mt > m_ref + RESCALE_LOG2;  // (first sub-tile: m_ref = -inf)
      const float al = bump ? __builtin_amdgcn_exp2f(m_ref - mt) : 1.f;
      if (bump) {
        l_run *= al;
        m_ref = mt;
      }
      float pv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = __builtin_amdgcn_exp2f(sc[i] - m_ref);
      l_run += xor32_sum(xor16_sum((pv[0] + pv[1]) + (pv[2] + pv[3])));
      ds_wr64(pimg + (16 * shb + fr) * 32 + 8 * fg, v2u32{pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3])});
      if (fg == 0) ds_wr32f(alph + (16 * shb + fr) * 4, al);
      const int anyb = (__builtin_amdgcn_read_exec() & __ballot(bump)) != 0;
      if (lane == 0) ds_wr32f(alph + QMAX * 4 + shb * 4, __int_as_float(anyb));
      lgkm0();
    }
    XSTAMP(11 + 8 * t);
    raw_barrier();  // C: P and the rescale factors published
    XSTAMP(12 + 8 * t);
    // 3. z = alpha z + P e over this wave's channels on v_mfma_f32_32x32x16_bf16: A = P [query l&31][frames
    //    8(l>>5) ..], B = e [frames 8(l>>5) ..][channel l&31] by two transposed reads of this wave's own pieces
    //    (group g = l>>4: frames 8hh + 4j' + q for lane 4q+p, channels 16(g&1) + 4p .. of the 32-channel block)
    bf16x8 pa = ds_rd128(pimg + (lane & 31) * 32 + 16 * (lane >> 5));
    int rescale = 0;
#pragma unroll
    for (int hb = 0; hb < HB; ++hb) rescale |= __float_as_int(ds_rd32f(alph + QMAX * 4 + hb * 4));
    v2u32 bt[KS][2];
    {
      const char* own = sl + wave * WREG;
      const int hh = lane >> 5, g = (lane >> 4) & 1, q = (lane & 15) >> 2, pp = lane & 3;
      const int cc = 2 * g + (pp >> 1);
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int r = 8 * hh + 4 * h2 + q;
          bt[k][h2] = ds_tr64(own + k * 1024 + r * 64 + ((cc ^ ((r >> 1) & 3)) << 4) + 8 * (pp & 1));
        }
    }
    lgkm0();
    tie(pa);
    tie(rescale);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      tie(bt[k][0]);
      tie(bt[k][1]);
    }
    if (__builtin_amdgcn_readfirstlane(rescale)) {  // wave-uniform, rare after the first sub-tile
      f32x4 av[4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) av[g4] = *reinterpret_cast<const f32x4*>(alph + (8 * g4 + 4 * (lane >> 5)) * 4);
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int r = 0; r < 16; ++r) zacc[k][r] *= av[r >> 2][r & 3];
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const v4u32 w = {bt[k][0][0], bt[k][0][1], bt[k][1][0], bt[k][1][1]};
      zacc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, w), zacc[k], 0, 0, 0);
    }
    XSTAMP(13 + 8 * t);
  }
  XSTAMP(2);

  // 4. publish the chunk's partials write-through: z (queries x D, f32) transposed through LDS (the ring is
  //    free) so that every store is a whole 16-B piece of a query row; (max, sum) per query
  __syncthreads();
  float* zt = reinterpret_cast<float*>(lds);  // [Q][D]
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (j < Q) zt[j * D + ch0 + 32 * k + (lane & 31)] = zacc[k][r];
    }
  __syncthreads();
  bf16_t* zpb = p.zp + (int64_t)blockIdx.x * QMAX * D;
  if (KW_XENC_LAB != 1)
    for (int idx = tid; idx < Q * (D >> 3); idx += NW * 64) {  // 8 channels (16 B of bf16) per store
      const f32x4 lo = reinterpret_cast<const f32x4*>(zt)[2 * idx], hi = reinterpret_cast<const f32x4*>(zt)[2 * idx + 1];
      st16_sc1(zpb + 8 * idx, v4u32{pack_bf16x2(lo[0], lo[1]), pack_bf16x2(lo[2], lo[3]), pack_bf16x2(hi[0], hi[1]),
                                    pack_bf16x2(hi[2], hi[3])});
    }
  if (swave && shalf == 0 && fg == 0 && 16 * shb + fr < Q) {  // the softmax state of query 16 shb + fr
    float* mlj = p.ml + ((int64_t)blockIdx.x * QMAX + 16 * shb + fr) * 2;
    __hip_atomic_store(mlj, m_ref, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mlj + 1, l_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  XSTAMP(3);
  __syncthreads();
  XSTAMP(4);
  // 5. item barrier: every chunk of item b has published
  if (p.nch > 1) {
    if (tid == 0) {
      __hip_atomic_fetch_add(p.cnt + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int n = 0, ok = 1;
      while (__hip_atomic_load(p.cnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p.nch) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > SPIN_MAX) {
          ok = 0;
          break;
        }
      }
      if (!ok) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  XSTAMP(5);
  // 6. merge: this workgroup finalises channels [D c / nch, D (c+1) / nch) of every query, chunks in order
  const int cb0 = 8 * (((D >> 3) * c) / p.nch), cb1 = 8 * (((D >> 3) * (c + 1)) / p.nch);  // whole 8-channel groups
  const float* mlb = p.ml + (int64_t)b * p.nch * QMAX * 2;
  if (tid < Q) {
    float mk[NCHMAX], M = -INFINITY;
#pragma unroll
    for (int k = 0; k < NCHMAX; ++k) {
      mk[k] = k < p.nch ? __hip_atomic_load(mlb + (k * QMAX + tid) * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -INFINITY;
      M = fmaxf(M, mk[k]);
    }
    float L = 0.f, f[NCHMAX];
#pragma unroll
    for (int k = 0; k < NCHMAX; ++k) {
      f[k] = k < p.nch ? __builtin_amdgcn_exp2f(mk[k] - M) : 0.f;  // (chunk maxima in the log2 domain)
      if (k < p.nch)
        L = fmaf(__hip_atomic_load(mlb + (k * QMAX + tid) * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), f[k], L);
    }
    const float inv = 1.f / L;
#pragma unroll
    for (int k = 0; k < NCHMAX; ++k) wts[k * QMAX + tid] = f[k] * inv;
  }
  __syncthreads();
  const int cw8 = (cb1 - cb0) >> 3;
  const bf16_t* zpi = p.zp + (int64_t)b * p.nch * QMAX * D;
  const int nit = KW_XENC_LAB == 1 ? 0 : Q * cw8;
  for (int idx0 = tid; idx0 < nit; idx0 += 2 * NW * 64) {  // two 8-channel pieces per thread in flight
    v4u32 v[2][NCHMAX];
    int jj[2], cc[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int idx = min(idx0 + r * NW * 64, nit - 1);
      jj[r] = idx / cw8;
      cc[r] = cb0 + 8 * (idx - jj[r] * cw8);
#pragma unroll
      for (int k = 0; k < NCHMAX; ++k) v[r][k] = ld16_sc1(zpi + ((int64_t)min(k, p.nch - 1) * QMAX + jj[r]) * D + cc[r]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
      for (int k = 0; k < NCHMAX; ++k) tie(v[r][k]);
      if (idx0 + r * NW * 64 >= nit) continue;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NCHMAX; ++k) {
        const float w = k < p.nch ? wts[k * QMAX + jj[r]] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] = fmaf(__uint_as_float(v[r][k][e] << 16), w, acc[2 * e]);
          acc[2 * e + 1] = fmaf(__uint_as_float(v[r][k][e] & 0xffff0000u), w, acc[2 * e + 1]);
        }
      }
      *reinterpret_cast<uint4*>(p.z + (qrow0 + jj[r]) * D + cc[r]) =
          make_uint4(pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
                     pack_bf16x2(acc[6], acc[7]));
    }
  }
  XSTAMP(6);
  // 7. departure: the last chunk of the item resets the counters for the next launch
  if (p.nch > 1) {
    __syncthreads();
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(p.dep + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == p.nch - 1) {
        __hip_atomic_store(p.cnt + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p.dep + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

int device_cus_x() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  return ncu;
}

// chunks per item: fill the CUs with one workgroup each (grid <= CUs keeps every chunk of an item resident)
int chunks_for(int64_t B) {
  const int64_t n = device_cus_x() / (B > 0 ? B : 1);
  return (int)(n < 1 ? 1 : (n > NCHMAX ? NCHMAX : n));
}

size_t hdr_bytes(int64_t B) { return (size_t)((2 * B + 1) * sizeof(int) + 255) / 256 * 256; }

constexpr int LDS_MAX = 160 * 1024;

// dynamic LDS: the ring + score partials + P image + rescale factors, or the partial-transpose image of
// Q query rows if larger, then the merge weights; sets p.wts_off
template <int NW, int KS>
size_t lds_bytes(XaP& p) {
  const size_t loop = (size_t)NBUF * NW * KS * 1024 + HB * 64 * 16 + QMAX * 32 + QMAX * 4 + HB * 4;
  const size_t zt = (size_t)p.Q * p.D * 4;
  p.wts_off = (int)(((loop > zt ? loop : zt) + 15) / 16 * 16);
  return (size_t)p.wts_off + NCHMAX * QMAX * 4;
}

template <int NW, int KS>
hipError_t launch_x(XaP p, int grid, hipStream_t s) {
  const size_t shm = lds_bytes<NW, KS>(p);
  if (shm > (size_t)LDS_MAX) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&xattn_enc_kernel<NW, KS>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((xattn_enc_kernel<NW, KS>), dim3((unsigned)grid), dim3(NW * 64), shm, s, p);
  return hipGetLastError();
}

}  // namespace

#if KW_XENC_STAMPS
extern "C" int kw_lab_xenc_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xenc_stamps), sizeof(g_xenc_stamps)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" size_t kw_cross_attn_enc_workspace(int64_t B, int64_t D) {
  if (B <= 0 || D <= 0) return 0;
  const int64_t blocks = B * chunks_for(B);
  return hdr_bytes(B) + (size_t)blocks * QMAX * 2 * sizeof(float) + (size_t)blocks * QMAX * D * sizeof(bf16_t);
}

extern "C" int kw_cross_attn_enc(const void* enc, int64_t B, int64_t S, int64_t D, const void* u, int64_t q_len,
                                 int64_t H, void* z, void* workspace, size_t ws_bytes, kw_stream_t stream) {
  if (!enc || !u || !z || !workspace || B <= 0 || S <= 0 || q_len <= 0 || H <= 0 || H > QMAX || (uintptr_t)enc % 16 ||
      (uintptr_t)u % 16 || (uintptr_t)z % 16)
    return kw_set_error_msg(KW_EINVAL, "kw_cross_attn_enc: invalid arguments (16-B aligned pointers, 1 <= H <= 32)");
  if (ws_bytes < kw_cross_attn_enc_workspace(B, D))
    return kw_set_error_msg(KW_EINVAL, "kw_cross_attn_enc: needs a zero-filled workspace of kw_cross_attn_enc_workspace()");
  const bool d_ok = D == 1280 || D == 1024 || D == 768 || D == 512 || D == 384;
  if (!d_ok) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_cross_attn_enc: d_model must be 384, 512, 768, 1024 or 1280");
  XaP p{};
  p.enc = (const bf16_t*)enc;
  p.S = (int)S;
  p.D = (int)D;
  p.H = (int)H;
  p.u = (const bf16_t*)u;
  p.z = (bf16_t*)z;
  p.q_len = (int)q_len;
  p.nch = chunks_for(B);
  p.nst = (int)((S + SUB - 1) / SUB);
  if (p.nch > p.nst) p.nch = p.nst;
  int* hdr = (int*)workspace;
  p.cnt = hdr;
  p.dep = hdr + B;
  p.err = hdr + 2 * B;
  p.ml = (float*)((char*)workspace + hdr_bytes(B));
  p.zp = reinterpret_cast<bf16_t*>(p.ml + (size_t)B * chunks_for(B) * QMAX * 2);
  const int grid = (int)(B * p.nch);
  const int rows = QMAX / (int)H;  // decode rows per launch (one K/V-free pass over e serves them all)
  hipStream_t s = (hipStream_t)stream;
  for (int64_t q0 = 0; q0 < q_len; q0 += rows) {
    p.qi0 = (int)q0;
    p.Q = (int)((q_len - q0 < rows ? q_len - q0 : rows) * H);
    hipError_t e;
    switch (D) {
      case 1280: e = launch_x<8, 5>(p, grid, s); break;
      case 1024: e = launch_x<8, 4>(p, grid, s); break;
      case 768: e = launch_x<8, 3>(p, grid, s); break;
      case 512: e = launch_x<8, 2>(p, grid, s); break;
      default: e = launch_x<4, 3>(p, grid, s); break;
    }
    if (e != hipSuccess) return kw_set_error(e);
  }
  return KW_OK;
}
