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
//  * gemm256_kernel: 256x256x64 ping-pong for the large encoder GEMMs (see its header below).
//  (decode-step skinny linears: declin.hip)
// Shared epilogues: bias, exact GELU, column scale (q * head_dim^-0.5, modeling_whisper.py:309),
// row-periodic add (encoder positions, :621-624), residual add into the f32 stream, head-split store.
#include <stdlib.h>

#include "gemm_common.h"

// development hook (tools/lab/gemm_lab.hip defines it to record s_memtime stamps); no-op here
#ifndef KW_GEMM_GM
#define KW_GEMM_GM 4  // row tiles per group in gemm256's tile order (1 = row-major)
#endif

#ifndef KW_GEMM_STAMP
#define KW_GEMM_STAMP(slot)
#endif

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
// bf16 256x256x64 ping-pong (encoder GEMMs, cross-K/V projection)
//
// 8 waves in two groups of four (one wave of each group per SIMD).  Group g owns output rows
// g*128..+128; wave q of a group owns columns q*64..+64 (8x4 tiles of v_mfma_f32_16x16x32_bf16,
// 128 accumulator registers).  The groups run one barrier apart, so on every SIMD one wave issues its
// LDS fragment reads while the other runs its 64-MFMA cluster.  LDS holds two K-tile buffers of
// 64 KB (A image + W image, 256 rows x 128 B, XOR-swizzled on the SOURCE address so the lane-linear
// global_load_lds image reads conflict-free).  Group 0 stages A, group 1 stages W; every staged tile
// has two barrier slots to land and is retired by the issuing wave's vmcnt before the barrier that
// precedes its first read (raw s_barrier: no implicit vmcnt(0) drain).
//
// Slot s = interval between two consecutive hardware barriers.  Slot 2t: group 0 reads tile t,
// group 1 multiplies tile t-1.  Slot 2t+1: group 0 multiplies tile t, group 1 reads tile t.  Every
// reader drains its LDS reads (lgkmcnt(0)) before the barrier that ends its read slot.  Group 0
// stages A of tile t+1 in slot 2t (tile t-1's buffer, last read in slot 2t-1) and retires it at the end
// of slot 2t+1; group 1 stages W of tile t+2 in slot 2t+1 after its own reads of tile t (group 0 read
// tile t in slot 2t) and retires it at the end of slot 2t+3.  Both are read from slot 2t+2 / 2t+4 on.
//
// Epilogue: each wave stages its 128x64 f32 results through a private 17 KB LDS region (64 rows at a
// time, 272-B padded rows: conflict-free b32 writes) and stores 16-B row pieces (4 f32 / 8 bf16), so
// every wave store instruction covers 4 (f32) or 8 (bf16) rows x 64 contiguous columns.
// ------------------------------------------------------------------------------------------------
constexpr int PB = 256, PK = 64;
constexpr int P_OP = PB * PK * 2;     // 32 KB: one operand image of one K-tile
constexpr int P_BUF = 2 * P_OP;       // 64 KB
constexpr int P_LDS = 2 * P_BUF;      // 128 KB of K-tile buffers
constexpr int P_EROW = 72;            // epilogue staging row stride (floats): 4 rows of a pass 16 banks apart
constexpr int P_EPI = 8 * P_EROW * 4; // per-wave epilogue staging region: 8 rows x 64 f32 (+pad)
constexpr int P_BIAS = PB * 4;        // the tile's 256 bias values
constexpr int P_LDS_ALLOC = P_LDS + 8 * P_EPI + P_BIAS;  // 147.5 KB

// Epilogue staging reads as inline asm: the compiler cannot tell them apart from the next tile's
// in-flight LDS-DMA targets and would put an s_waitcnt vmcnt(0) -- which also waits for every store
// already issued -- in front of each one, serialising the store stream.  The staging region never
// receives LDS-DMA, so only the wave's own ds_writes (in order) must precede the reads.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// issue one 16-B staging read; lds_wait(v) (s_waitcnt lgkmcnt(0) tied to v) must precede any use of v
__device__ __forceinline__ void lds_issue_read(const float* p, f32x4& v) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
}
__device__ __forceinline__ void lds_wait(f32x4& v) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v)); }

__device__ __forceinline__ void pp_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

template <int EPI, typename TC>
__global__ __launch_bounds__(512) void gemm256_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wq = wave & 3;

  // Persistent walk: the tiles are cut into 8 contiguous runs (one per XCD, bid & 7); the WGs of an XCD
  // take its run's tiles round-robin, so the tiles an XCD holds at once are neighbours sharing A rows.
  const int tiles_n = p.N / PB;
  const int tiles_m = (p.M + PB - 1) / PB;
  const int nwg = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int run0 = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int run_len = q8 + (xcd < r8 ? 1 : 0);
  const int per = (G >> 3) + (xcd < (G & 7) ? 1 : 0);  // WGs on this XCD
  int pos = loc;
  if (pos >= run_len) return;

  const int nk = p.K / PK;
  const char* sbase = grp == 0 ? reinterpret_cast<const char*>(p.A) : reinterpret_cast<const char*>(p.W);
  uint32_t soff[8];
  int m0 = 0, n0 = 0;
  // staging sources: group 0 -> A rows m0.., group 1 -> W rows n0..; 8 x 1 KB glds per wave per K-tile
  auto set_tile = [&](int idx, int lane) {
    const int wg = run0 + idx;
    // grouped order: KW_GEMM_GM row tiles walk the columns together, so the ~32 tiles an XCD holds at
    // once span GM row blocks x (32 / GM) column blocks and share both operands in its L2
    const int per_group = KW_GEMM_GM * tiles_n;
    const int gidx = wg / per_group;
    const int first_m = gidx * KW_GEMM_GM;
    const int gm = min(KW_GEMM_GM, tiles_m - first_m);
    const int rr = wg - gidx * per_group;
    const int tm = first_m + rr % gm, tn = rr / gm;
    m0 = tm * PB;
    n0 = tn * PB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 8 * (wq * 8 + i) + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (grp == 0) {
        const int m = min(m0 + r, p.M - 1);
        soff[i] = (uint32_t)((row_off(m, p.a_rpb, p.a_bs, p.lda) + c * 8) * 2);
      } else {
        soff[i] = (uint32_t)(((int64_t)(n0 + r) * p.K + c * 8) * 2);
      }
    }
  };
  auto stage = [&](int t, int buf) {
    char* dst = smem + buf * P_BUF + grp * P_OP + wq * 8 * 1024;
    const char* src = sbase + (int64_t)t * (PK * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i) glds16(src + soff[i], dst + i * 1024);
  };
  float* bias_lds = reinterpret_cast<float*>(smem + P_LDS + 8 * P_EPI);
  // prologue loads of a tile: A (group 0) / W (group 1) of K-tile 0, W of K-tile 1, the bias row (wave 0)
  auto prologue = [&]() {
    stage(0, 0);
    if (grp == 1 && nk > 1) stage(1, 1);
    if (wave == 0 && p.bias) glds16(p.bias + n0 + 4 * (tid & 63), reinterpret_cast<char*>(bias_lds));
  };
  // wait for what the first K-tile needs: every load but group 1's 8 pieces of K-tile 1 (issued after
  // K-tile 0), and -- when ``after`` stores were issued since -- those stores too (vmcnt is in order)
  auto prologue_wait = [&](bool stores_after) {
    const bool w1 = grp == 1 && nk > 1;
    if (stores_after) {
      if constexpr (EPI != KW_EPI_RESID && sizeof(TC) == 2) {
        if (w1) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // 16 epilogue stores + 8 W pieces
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else if constexpr (EPI != KW_EPI_RESID) {
        if (w1) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");  // 32 f32 stores + 8
        else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      if (w1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  // fragment read offsets (row = lane & 15 within a 16-row rep; the swizzle term (row >> 1) & 7 is per lane)
  const int swz = (lane & 15) >> 1;
  const int rd0 = (lane & 15) * 128 + (((0 * 4 + (lane >> 4)) ^ swz) << 4);
  const int rd1 = (lane & 15) * 128 + (((1 * 4 + (lane >> 4)) ^ swz) << 4);

  f32x4 acc[8][4];
  bf16x8 a[8][2], b[4][2];
  auto read_frags = [&](int buf) {
    const char* As = smem + buf * P_BUF + grp * 128 * 128;
    const char* Bs = smem + buf * P_BUF + P_OP + wq * 64 * 128;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      b[j][0] = *reinterpret_cast<const bf16x8*>(Bs + j * 2048 + rd0);
      b[j][1] = *reinterpret_cast<const bf16x8*>(Bs + j * 2048 + rd1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i][0] = *reinterpret_cast<const bf16x8*>(As + i * 2048 + rd0);
      a[i][1] = *reinterpret_cast<const bf16x8*>(As + i * 2048 + rd1);
    }
  };
  auto mma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b[j][ks], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // group 0's read slot: its 8 A pieces for tile t+1 interleaved one per 3 fragment reads (r05: the pieces issued
  // after all 24 reads left the slot longer; encoder 69.4-69.9 -> 68.8-69.0 ms, profiles/r05p_enc_ab.txt)
  auto read_stage = [&](int buf, int tt, bool do_stage) {
    const char* As = smem + buf * P_BUF + grp * 128 * 128;
    const char* Bs = smem + buf * P_BUF + P_OP + wq * 64 * 128;
    char* dst = smem + (buf ^ 1) * P_BUF + wq * 8 * 1024;
    const char* src = sbase + (int64_t)tt * (PK * 2);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (do_stage) glds16(src + soff[k], dst + k * 1024);
#pragma unroll
      for (int r = 3 * k; r < 3 * k + 3; ++r) {
        if (r < 8) b[r >> 1][r & 1] = *reinterpret_cast<const bf16x8*>(Bs + (r >> 1) * 2048 + ((r & 1) ? rd1 : rd0));
        else a[(r - 8) >> 1][(r - 8) & 1] = *reinterpret_cast<const bf16x8*>(As + ((r - 8) >> 1) * 2048 + (((r - 8) & 1) ? rd1 : rd0));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // The residual epilogue reads C and row_add reads a table: those loads would queue behind the next
  // tile's prologue (vmcnt is in order), so such launches issue the prologue after the epilogue.
  const bool overlap = EPI != KW_EPI_RESID && !p.row_add;
  set_tile(pos, lane);
  prologue();
  prologue_wait(false);

  [[maybe_unused]] int tcount = 0;  // tile counter for the lab stamps
  KW_GEMM_STAMP(0);
  for (;;) {
    // an opaque copy of the lane id per tile: keeps the epilogue's lane-derived addresses from being
    // hoisted out of the tile loop (they would stay live across the main loop and spill)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    pp_barrier();
    if (grp == 1) pp_barrier();  // the stagger
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    KW_GEMM_STAMP(1 + 3 * tcount);

    if (grp == 0) {
      for (int t = 0; t < nk; ++t) {
        const int buf = t & 1;
        read_stage(buf, t + 1, t + 1 < nk);  // + A of tile t+1 (its buffer's last reader finished in slot 2t-1)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();
        mma();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // A of tile t+1 landed
        pp_barrier();
      }
      pp_barrier();  // balances group 1's stagger barrier
    } else {
      // group 1 stages W of tile t+2 in its own read slot, after its reads of tile t drained: group 0 read
      // tile t one slot earlier, so the buffer is free; the W of tile t+1 (issued one read slot earlier)
      // must have landed before this slot's barrier: vmcnt(8) leaves only the 8 just-issued pieces.
      for (int t = 0; t < nk; ++t) {
        const int buf = t & 1;
        read_frags(buf);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (t + 2 < nk) {
          stage(t + 2, buf);
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        pp_barrier();
        mma();
        pp_barrier();
      }
    }
    // every wave passed the last barrier: the K-tile buffers are free, every glds retired.  Pull this
    // tile's bias out of LDS before the next prologue overwrites it.
    KW_GEMM_STAMP(2 + 3 * tcount);
    const int tm0 = m0, tn0 = n0;
    const bool full = tm0 + PB <= p.M;
    constexpr int VEC = (EPI != KW_EPI_RESID && sizeof(TC) == 2) ? 8 : 4;
    constexpr int LPR = 64 / VEC;  // lanes per 64-column row
    constexpr int RPI = 64 / LPR;  // rows per store instruction
    const int cq = ln % LPR;     // this lane's VEC-column group within the wave's 64 columns
    const int n = tn0 + wq * 64 + VEC * cq;
    float cb[VEC];
#pragma unroll
    for (int e = 0; e < VEC; e += 4) {
      const float4 b4 = p.bias ? *reinterpret_cast<const float4*>(bias_lds + wq * 64 + VEC * cq + e)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
      cb[e] = b4.x; cb[e + 1] = b4.y; cb[e + 2] = b4.z; cb[e + 3] = b4.w;
    }
    pos += per;
    const bool more = pos < run_len;
    if (more && overlap) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();  // every wave holds its bias before wave 0 restages the bias row
      set_tile(pos, ln);
      prologue();
    }

    // epilogue: each wave stages its 128x64 results 8 rows at a time (rows 4g + 2h + {0,1} of a 16-row
    // tile, LDS row 2g + {0,1}) through a private region beside the K-tile buffers, then stores 16-B row
    // pieces (8 bf16 / 4 f32): one (bf16) or two (f32) store instructions per pass.
    float* ep = reinterpret_cast<float*>(smem + P_LDS + wave * P_EPI);
    // per-column affine: v = acc * cmul + cadd (no GELU: bias and column scale folded), or
    // v = gelu(acc + cadd) * cmul
    float cmul[VEC], cadd[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      cmul[e] = n + e < p.scale_cols ? p.scale : 1.f;
      cadd[e] = p.gelu ? cb[e] : cb[e] * cmul[e];
    }
    // Row -> element offset.  A 256-row tile meets at most one batch boundary when a batch holds >= 256
    // rows (the encoder's 1500 / 3000): rows below ``bnd`` continue from rb0, the rest from rb1.
    // Smaller batches (tests) take the general division per row.
    int64_t coff = n;
    const int rpb = EPI == KW_EPI_HEADSPLIT ? p.hs_seq : (int)p.c_rpb;
    int64_t rstride, bstride;
    if constexpr (EPI == KW_EPI_HEADSPLIT) {
      const int nb = p.M / p.hs_seq;
      const int width = p.hs_heads * p.hs_hd;
      const int part = n / width, rem = n - part * width;
      const int h = rem / p.hs_hd, d = rem - h * p.hs_hd;
      coff = ((int64_t)part * nb * p.hs_heads + h) * (int64_t)p.hs_seq * p.hs_hd + d;
      rstride = p.hs_hd;
      bstride = (int64_t)p.hs_heads * p.hs_seq * p.hs_hd;
    } else {
      rstride = p.ldc;
      bstride = p.c_bs;
    }
    const bool linear = rpb >= PB;
    const int b0 = tm0 / rpb;
    const int bnd = (b0 + 1) * rpb;
    const int64_t rb0 = (int64_t)b0 * bstride + (int64_t)(tm0 - b0 * rpb) * rstride + coff;
    const int64_t rb1 = (int64_t)(b0 + 1) * bstride + coff;
    auto row_offset = [&](int m) -> int64_t {
      if (linear) return m < bnd ? rb0 + (int64_t)(m - tm0) * rstride : rb1 + (int64_t)(m - bnd) * rstride;
      const int bb = m / rpb;
      return (int64_t)bb * bstride + (int64_t)(m - bb * rpb) * rstride + coff;
    };
    if constexpr (EPI == KW_EPI_RESID) {
      // Residual add C(f32) += acc + bias: the C reads of 16-row block i+1 are issued before block i's
      // staging, adds and stores, so each block waits on loads already in flight instead of one dependent
      // round trip per row piece (28 -> 16 us per 256x256 tile at 48000 x 1280; a deeper ring spills).
      constexpr int NP = 2 * (8 / RPI);  // row pieces per lane per 16-row block
      f32x4 res[2][NP];
      int64_t roff[2][NP];
      auto issue = [&](int i, f32x4* r, int64_t* o) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int q = 0; q < 8 / RPI; ++q) {
            const int lr = RPI * q + ln / LPR;
            const int m = tm0 + grp * 128 + 16 * i + 4 * (lr >> 1) + 2 * hh + (lr & 1);
            const int pi = hh * (8 / RPI) + q;
            o[pi] = row_offset(min(m, p.M - 1));
            r[pi] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.C) + o[pi]);
          }
      };
      issue(0, res[0], roff[0]);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i + 1 < 8) issue(i + 1, res[(i + 1) & 1], roff[(i + 1) & 1]);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2)
              ep[(2 * (ln >> 4) + r2) * P_EROW + 16 * j + (ln & 15)] = acc[i][j][2 * hh + r2];
#pragma unroll
          for (int q = 0; q < 8 / RPI; ++q) {
            const int lr = RPI * q + ln / LPR;
            const int m = tm0 + grp * 128 + 16 * i + 4 * (lr >> 1) + 2 * hh + (lr & 1);
            const int pi = hh * (8 / RPI) + q;
            f32x4 v4;
            lds_issue_read(ep + lr * P_EROW + VEC * cq, v4);
            lds_wait(v4);
            if (m >= p.M) continue;
            const f32x4 o = res[i & 1][pi];
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.C) + roff[i & 1][pi]) =
                f32x4{o[0] + (v4[0] + cb[0]), o[1] + (v4[1] + cb[1]), o[2] + (v4[2] + cb[2]), o[3] + (v4[3] + cb[3])};
          }
        }
      }
    } else
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r2 = 0; r2 < 2; ++r2)
            ep[(2 * (ln >> 4) + r2) * P_EROW + 16 * j + (ln & 15)] = acc[i][j][2 * hh + r2];
#pragma unroll
        for (int q = 0; q < 8 / RPI; ++q) {
          const int lr = RPI * q + ln / LPR;  // LDS row 0..7
          const int m = tm0 + grp * 128 + 16 * i + 4 * (lr >> 1) + 2 * hh + (lr & 1);
          f32x4 v4[VEC / 4];
          lds_issue_read(ep + lr * P_EROW + VEC * cq, v4[0]);
          if constexpr (VEC == 8) lds_issue_read(ep + lr * P_EROW + VEC * cq + 4, v4[1]);
          const int64_t off = row_offset(m);
          lds_wait(v4[0]);
          if constexpr (VEC == 8) lds_wait(v4[1]);
          float v[VEC];
#pragma unroll
          for (int e = 0; e < VEC; ++e) v[e] = v4[e >> 2][e & 3];
          if (m >= p.M) continue;
          if constexpr (EPI == KW_EPI_RESID) {
            float4* c = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + off);
            float4 o = *c;
            o.x += v[0] + cb[0]; o.y += v[1] + cb[1]; o.z += v[2] + cb[2]; o.w += v[3] + cb[3];
            *c = o;
          } else {
            if (p.gelu) {
#pragma unroll
              for (int e = 0; e < VEC; ++e)
                v[e] = (sizeof(TC) == 2 ? gelu_bf16out(v[e] + cadd[e]) : gelu_erf(v[e] + cadd[e])) * cmul[e];
            } else {
#pragma unroll
              for (int e = 0; e < VEC; ++e) v[e] = fmaf(v[e], cmul[e], cadd[e]);
            }
            if (p.row_add) {
              const float* ra = p.row_add + (int64_t)(m % p.row_add_period) * p.N + n;
#pragma unroll
              for (int e = 0; e < VEC; e += 4) {
                const float4 r4 = *reinterpret_cast<const float4*>(ra + e);
                v[e] += r4.x; v[e + 1] += r4.y; v[e + 2] += r4.z; v[e + 3] += r4.w;
              }
            }
            if constexpr (sizeof(TC) == 4) {
              *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + off) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
              uint4 o;
              o.x = pack_bf16x2(v[0], v[1]);
              o.y = pack_bf16x2(v[2], v[3]);
              o.z = pack_bf16x2(v[4], v[5]);
              o.w = pack_bf16x2(v[6], v[7]);
              // non-temporal where the consumer is compute-bound (head-split q/k/v and cross K/V for the attention,
              // fc1's GELU output for fc2): the tile's 128 KB of stores then do not evict the operand panels the next
              // tiles re-read (tools/gemm_bench.py, r03z: QKV 500 -> 465-484, fc1 621 -> 590, cross K/V 9.3 -> 8.2 ms);
              // the out-proj / fc2 deltas stay cacheable for the HBM-bound LayerNorm that reads them next
              const bool nt = EPI == KW_EPI_HEADSPLIT || p.gelu;
              typedef __attribute__((ext_vector_type(4))) unsigned int nt_u4;
              if (nt)
                __builtin_nontemporal_store(nt_u4{o.x, o.y, o.z, o.w}, reinterpret_cast<nt_u4*>(reinterpret_cast<bf16_t*>(p.C) + off));
              else
                *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.C) + off) = o;
            }
          }
        }
      }
    }
    KW_GEMM_STAMP(3 + 3 * tcount);
    ++tcount;
    if (!more) break;
    if (overlap) {
      prologue_wait(full);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      pp_barrier();  // every wave read its bias
      set_tile(pos, ln);
      prologue();
      prologue_wait(false);
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

template <int EPI, typename TC>
hipError_t launch256_one(const GemmP& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_kernel<EPI, TC>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, P_LDS_ALLOC);
    if (e != hipSuccess) return e;
    attr = true;
  }
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  const int nwg = ((p.M + PB - 1) / PB) * (p.N / PB);
  const int grid = nwg < ncu ? nwg : ncu;  // persistent: one 147.5-KB-LDS workgroup per CU
  hipLaunchKernelGGL((gemm256_kernel<EPI, TC>), dim3(grid), dim3(512), P_LDS_ALLOC, s, p);
  return hipGetLastError();
}

template <typename TC>
hipError_t launch256(const GemmP& p, int epi, hipStream_t s) {
  switch (epi) {
    case KW_EPI_STORE: return launch256_one<KW_EPI_STORE, TC>(p, s);
    case KW_EPI_RESID: return launch256_one<KW_EPI_RESID, float>(p, s);
    default: return launch256_one<KW_EPI_HEADSPLIT, TC>(p, s);
  }
}

// 256x256 ping-pong for the big GEMMs (the 128x128 kernel for shapes it does not take).
bool use256(const kw_gemm_args* a) {
  // vector epilogue: ldc, batch strides, head_dim in whole 16-B pieces, the C base 16-B aligned
  const int vec = (a->c_dtype == KW_DT_F32) ? 4 : 8;  // 16-B pieces: 4 f32 / 8 bf16 columns
  const bool aligned = a->ldc % vec == 0 && a->c_batch_stride % vec == 0 &&
                       (a->hs_head_dim <= 0 || a->hs_head_dim % vec == 0) && ((uintptr_t)a->C % 16) == 0 &&
                       ((uintptr_t)a->row_add % 16) == 0;
  return aligned && a->N % PB == 0 && a->M >= 4 * PB;
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
    if (use256(a))
      e = a->c_dtype == KW_DT_F32 ? launch256<float>(p, a->epilogue, s) : launch256<bf16_t>(p, a->epilogue, s);
    else
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
