// Lab (r03): how fast can the decode cross-attention's K/V bytes stream on gfx950, by kernel structure?
// Pure streaming probes over the production layout K/V [B][H][S][64] bf16 (no softmax): each workgroup reads
// its bytes and folds them into one word (so the loads cannot be dropped), written to out[wg].
//   reg   : grid (B*H, ns), 256 threads, every 16-B piece of the chunk's K and V by nt register loads,
//           all in flight at once (the production kernel's V side), PER = pieces per lane per tensor
//   dma   : the same grid, K and V by LDS-DMA nt (global_load_lds_dwordx4), LDS bytes per WG = 64 KB
//   kdma  : K by LDS-DMA, V by registers (the production kernel's load structure)
//   loop  : grid = nwg persistent workgroups walking (row, chunk) items, two items' loads in flight
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC tools/lab/xa_lab.hip -o tools/lab/libxa_lab.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

namespace {
constexpr int HD = 64;

__device__ __forceinline__ void glds16_nt(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 2);
}
__device__ __forceinline__ u32x4 ld_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// keys of a chunk: 8 lanes per 128-B key row, 32 rows per 256-thread pass; PER passes
template <int PER>
__global__ __launch_bounds__(256) void reg_kernel(const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc, int S,
                                                  int chunk, uint32_t* __restrict__ out) {
  const int row = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, sub = tid & 7, slot = tid >> 3;
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);
  const bf16_t* kb = kc + (int64_t)row * S * HD;
  const bf16_t* vb = vc + (int64_t)row * S * HD;
  u32x4 kr[PER], vr[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) kr[j] = ld_nt(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
#pragma unroll
  for (int j = 0; j < PER; ++j) vr[j] = ld_nt(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) x ^= fold(kr[j]) ^ fold(vr[j]);
  if (x == 0x12345678u) out[row * gridDim.y + split] = x;  // practically never: keeps the loads live
}

template <int PER>
__global__ __launch_bounds__(256) void dma_kernel(const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc, int S,
                                                  int chunk, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char kv[2 * PER * 4 * 1024];
  const int row = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);
  const bf16_t* kb = kc + (int64_t)row * S * HD;
  const bf16_t* vb = vc + (int64_t)row * S * HD;
#pragma unroll
  for (int j = 0; j < PER; ++j) glds16_nt(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8, kv + (4 * j + wave) * 1024);
#pragma unroll
  for (int j = 0; j < PER; ++j)
    glds16_nt(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8, kv + PER * 4096 + (4 * j + wave) * 1024);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 2 * PER; ++j) x ^= fold(*reinterpret_cast<const u32x4*>(kv + (4 * j + wave) * 1024 + lane * 16));
  if (x == 0x12345678u) out[row * gridDim.y + split] = x;
}

template <int PER>
__global__ __launch_bounds__(256) void kdma_kernel(const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc, int S,
                                                   int chunk, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char kv[PER * 4 * 1024];
  const int row = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);
  const bf16_t* kb = kc + (int64_t)row * S * HD;
  const bf16_t* vb = vc + (int64_t)row * S * HD;
#pragma unroll
  for (int j = 0; j < PER; ++j) glds16_nt(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8, kv + (4 * j + wave) * 1024);
  u32x4 vr[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) vr[j] = ld_nt(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) x ^= fold(*reinterpret_cast<const u32x4*>(kv + (4 * j + wave) * 1024 + lane * 16)) ^ fold(vr[j]);
  if (x == 0x12345678u) out[row * gridDim.y + split] = x;
}

// persistent: workgroup w takes items w, w + nwg, ... (item = row * ns + split); the next item's loads are
// issued before the current one is folded (two items in flight)
template <int PER>
__global__ __launch_bounds__(256) void loop_kernel(const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc, int S,
                                                   int chunk, int ns, int n_items, uint32_t* __restrict__ out) {
  const int tid = threadIdx.x, sub = tid & 7, slot = tid >> 3;
  u32x4 kr[2][PER], vr[2][PER];
  auto issue = [&](int item, int buf) {
    const int row = item / ns, split = item - row * ns;
    const int k0 = split * chunk, k1 = min(S, k0 + chunk);
    const bf16_t* kb = kc + (int64_t)row * S * HD;
    const bf16_t* vb = vc + (int64_t)row * S * HD;
#pragma unroll
    for (int j = 0; j < PER; ++j) kr[buf][j] = ld_nt(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
#pragma unroll
    for (int j = 0; j < PER; ++j) vr[buf][j] = ld_nt(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
  };
  uint32_t x = 0;
  int item = blockIdx.x;
  if (item < n_items) issue(item, 0);
  int buf = 0;
  for (; item < n_items; item += gridDim.x) {
    const int nxt = item + gridDim.x;
    if (nxt < n_items) issue(nxt, buf ^ 1);
#pragma unroll
    for (int j = 0; j < PER; ++j) x ^= fold(kr[buf][j]) ^ fold(vr[buf][j]);
    buf ^= 1;
  }
  if (x == 0x12345678u) out[blockIdx.x] = x;
}

// pair streaming (csrc/attention.hip cross_attn_row_kernel's load structure, no softmax): one workgroup per row,
// NS chunks in order, three 8-register K / V sets in rotation (K(c+1) out before chunk c's fold, V(c+1) right
// after the K fold, K(c+2) after the V fold)
__device__ __forceinline__ void row_ld(const bf16_t* base, int k0, int k1, int slot, int sub, u32x4 (&r)[8]) {
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = ld_nt(base + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
  __builtin_amdgcn_sched_barrier(0);
}
template <int NS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void rowstream_kernel(
    const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc, int S, int chunk, uint32_t* __restrict__ out) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const bf16_t* kb = kc + (int64_t)row * S * HD;
  const bf16_t* vb = vc + (int64_t)row * S * HD;
  u32x4 r0[8], r1[8], r2[8];
  row_ld(kb, 0, min(S, chunk), slot, sub, r0);
  row_ld(vb, 0, min(S, chunk), slot, sub, r1);
  if (NS > 1) row_ld(kb, chunk, min(S, 2 * chunk), slot, sub, r2);
  uint32_t x = 0;
  auto step = [&](const int c, u32x4 (&rk)[8], u32x4 (&rv)[8]) __attribute__((always_inline)) {
    const int k0 = c * chunk, k1 = min(S, k0 + chunk);
#pragma unroll
    for (int j = 0; j < 8; ++j) x ^= fold(rk[j]);
    if (c + 1 < NS) row_ld(vb, k1, min(S, k1 + chunk), slot, sub, rk);
#pragma unroll
    for (int j = 0; j < 8; ++j) x ^= fold(rv[j]);
    if (c + 2 < NS) row_ld(kb, k0 + 2 * chunk, min(S, k0 + 3 * chunk), slot, sub, rv);
  };
#pragma unroll
  for (int c = 0; c < NS; c += 3) {
    step(c, r0, r1);
    if (c + 1 < NS) step(c + 1, r2, r0);
    if (c + 2 < NS) step(c + 2, r1, r2);
  }
  if (x == 0x12345678u) out[row] = x;
}
}  // namespace

extern "C" int xa_lab_run(int variant, int per, const void* k, const void* v, int rows, int S, int ns, int nwg, void* out,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int chunk = (S + ns - 1) / ns;
  const dim3 grid((unsigned)rows, (unsigned)ns);
  const bf16_t* kc = (const bf16_t*)k;
  const bf16_t* vc = (const bf16_t*)v;
  uint32_t* o = (uint32_t*)out;
#define KW_LAB_PER(KER, ...)                                                                    \
  switch (per) {                                                                                \
    case 2: hipLaunchKernelGGL(KER<2>, __VA_ARGS__); break;                                     \
    case 4: hipLaunchKernelGGL(KER<4>, __VA_ARGS__); break;                                     \
    case 8: hipLaunchKernelGGL(KER<8>, __VA_ARGS__); break;                                     \
    default: return 2;                                                                          \
  }
  if (chunk > 32 * per) return 3;  // each chunk covered by one pass of PER rows per lane group
  switch (variant) {
    case 0: KW_LAB_PER(reg_kernel, grid, dim3(256), 0, s, kc, vc, S, chunk, o); break;
    case 1: KW_LAB_PER(dma_kernel, grid, dim3(256), 0, s, kc, vc, S, chunk, o); break;
    case 2: KW_LAB_PER(kdma_kernel, grid, dim3(256), 0, s, kc, vc, S, chunk, o); break;
    case 3: KW_LAB_PER(loop_kernel, dim3((unsigned)nwg), dim3(256), 0, s, kc, vc, S, chunk, ns, rows * ns, o); break;
    case 4:
      if (ns != 6) return 5;
      hipLaunchKernelGGL(rowstream_kernel<6>, dim3((unsigned)rows), dim3(256), 0, s, kc, vc, S, chunk, o);
      break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

// ---------------------------------------------------------------------------------------------------------
// The production cross-attention DMA kernel (csrc/attention.hip cross_attn_dma_kernel, r03 granule combine)
// copied with stage switches, to find where its time beyond the pure stream goes.
//   MODE 0 production arithmetic + granule combine   1 no combine (partials written, never merged)
//   MODE 2 fold only (= kdma probe)                    3 as 0 with exp2 (log2e folded) + DPP wave sums
//   MODE 4 as 3, no mid-chunk barrier: each wave its own softmax partial, merged once at the end
#include "../../kotoba-whisper_amd/csrc/kw_common.h"
namespace xl {
constexpr int HD = 64;
constexpr float LOG2E = 1.4426950408889634f;
__device__ __forceinline__ u32x4 lds_rd16(const char* p) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p) : "memory");
  return v;
}
__device__ __forceinline__ void unpack8(u32x4 u, float v[8]) {
  const uint32_t w[4] = {u[0], u[1], u[2], u[3]};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ float dpp_wave_sum(float v) {  // ^1 ^2 ^4 ^8 then ^16 ^32 swaps (DPP, no LDS)
  v += kw_dpp<0xB1>(v);
  v += kw_dpp<0x4E>(v);
  v += kw_dpp<0x141>(v);
  v += kw_dpp<0x140>(v);
  return kw_swap32_sum(kw_swap16_sum(v));
}
__device__ __forceinline__ void put_g(unsigned long long* g, float v) {
  __hip_atomic_store(g, (1ull << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__global__ __launch_bounds__(256) void xa_kernel(const bf16_t* __restrict__ q, int H, const bf16_t* __restrict__ kc,
                                                 const bf16_t* __restrict__ vc, int S, int chunk,
                                                 unsigned long long* __restrict__ gran, bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char kv[32 * 1024];
  __shared__ float red[4][64];
  __shared__ float stat[16];
  const int row = blockIdx.x, split = blockIdx.y, ns = gridDim.y;
  const int h = row % H, b = row / H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = lane & 7, slot = wave * 8 + (lane >> 3);
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);
  const bf16_t* kb = kc + ((int64_t)b * H + h) * S * HD;
  const bf16_t* vb = vc + ((int64_t)b * H + h) * S * HD;
  u32x4 qraw;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qraw) : "v"(q + (int64_t)b * H * HD + h * HD + sub * 8) : "memory");
#pragma unroll
  for (int j = 0; j < 8; ++j) glds16_nt(kb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8, kv + (4 * j + wave) * 1024);
  u32x4 vr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) vr[j] = ld_nt(vb + (int64_t)min(k0 + slot + 32 * j, k1 - 1) * HD + sub * 8);
  asm volatile("s_waitcnt vmcnt(8)" : "+v"(qraw) :: "memory");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  u32x4 kr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) kr[j] = lds_rd16(kv + (4 * j + wave) * 1024 + lane * 16);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kr[0]), "+v"(kr[1]), "+v"(kr[2]), "+v"(kr[3]), "+v"(kr[4]), "+v"(kr[5]),
               "+v"(kr[6]), "+v"(kr[7]));
  if constexpr (MODE == 2) {
    uint32_t x = qraw[0];
#pragma unroll
    for (int j = 0; j < 8; ++j) x ^= fold(kr[j]) ^ fold(vr[j]);
    if (x == 0x12345678u) out[row] = 1;
    return;
  }
  float qv[8];
  unpack8(qraw, qv);
  if constexpr (MODE >= 3 && MODE < 5) {
#pragma unroll
    for (int i = 0; i < 8; ++i) qv[i] *= LOG2E;
  }
  float sc[8], mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float sj = 0.f;
    if constexpr (MODE >= 5) {  // packed bf16 dot products (v_dot2c_f32_bf16), then to log2 units
      typedef __attribute__((ext_vector_type(2))) __bf16 bf2;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        sj = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, qraw[i]), __builtin_bit_cast(bf2, kr[j][i]), sj, false);
      sj *= LOG2E;
    } else {
      float kf[8];
      unpack8(kr[j], kf);
#pragma unroll
      for (int i = 0; i < 8; ++i) sj = fmaf(qv[i], kf[i], sj);
    }
    sj = kw_sum8(sj);
    sc[j] = (k0 + slot + 32 * j < k1) ? sj : -INFINITY;
    mx = fmaxf(mx, sc[j]);
  }
  mx = wave_max(mx);
  float m;
  if constexpr (MODE >= 4) {
    m = mx;  // this wave's own reference (merged at the end)
  } else {
    if (lane == 0) stat[wave] = mx;
    __syncthreads();
    m = fmaxf(fmaxf(stat[0], stat[1]), fmaxf(stat[2], stat[3]));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float lsum = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float pj;
    if constexpr (MODE >= 3) pj = (k0 + slot + 32 * j < k1) ? __builtin_amdgcn_exp2f(sc[j] - m) : 0.f;
    else pj = (k0 + slot + 32 * j < k1) ? expf(sc[j] - m) : 0.f;
    lsum += pj;
    if constexpr (MODE >= 5) {  // two f32 lanes per v_pk_fma_f32
      typedef __attribute__((ext_vector_type(2))) float f2;
      const f2 pp = {pj, pj};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f2 vv = {__uint_as_float(vr[j][i] << 16), __uint_as_float(vr[j][i] & 0xffff0000u)};
        f2 a = {acc[2 * i], acc[2 * i + 1]};
        a = __builtin_elementwise_fma(pp, vv, a);
        acc[2 * i] = a.x;
        acc[2 * i + 1] = a.y;
      }
    } else {
      float vv[8];
      unpack8(vr[j], vv);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(pj, vv[i], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = kw_sum_hi(acc[i]);
  if constexpr (MODE >= 3) lsum = dpp_wave_sum(lsum) * 0.125f;
  else lsum = wave_sum(lsum) * 0.125f;
  if (lane < 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wave][lane * 8 + i] = acc[i];
  }
  if (lane == 0) {
    stat[4 + wave] = lsum;
    stat[8 + wave] = m;
  }
  __syncthreads();
  float l, o, mm;
  if constexpr (MODE >= 4) {
    mm = fmaxf(fmaxf(stat[8], stat[9]), fmaxf(stat[10], stat[11]));
    float f[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) f[w] = __builtin_amdgcn_exp2f(stat[8 + w] - mm);
    l = (stat[4] * f[0] + stat[5] * f[1]) + (stat[6] * f[2] + stat[7] * f[3]);
    o = tid < HD ? (red[0][tid] * f[0] + red[1][tid] * f[1]) + (red[2][tid] * f[2] + red[3][tid] * f[3]) : 0.f;
  } else {
    mm = m;
    l = (stat[4] + stat[5]) + (stat[6] + stat[7]);
    o = tid < HD ? (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]) : 0.f;
  }
  bf16_t* orow = out + (int64_t)b * H * HD + h * HD;
  constexpr int G = HD + 2;
  unsigned long long* gr = gran + (int64_t)row * ns * G;
  if (MODE == 1 || split != ns - 1) {
    unsigned long long* w = gr + (int64_t)split * G;
    if (tid < HD) put_g(w + 2 + tid, o);
    if (tid == 0) {
      put_g(w, mm);
      put_g(w + 1, l);
    }
    if (MODE == 1 && split == ns - 1 && tid < HD) orow[tid] = f2bf(o / l);
    return;
  }
  if (tid >= HD) return;
  float ms[8], ls[8], os[8];
  for (int it = 0;; ++it) {
    unsigned long long x[21];
#pragma unroll
    for (int qq = 0; qq < 7; ++qq) {
      const unsigned long long* gq = gr + min(qq, ns - 2) * G;
      x[3 * qq] = __hip_atomic_load(gq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x[3 * qq + 1] = __hip_atomic_load(gq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      x[3 * qq + 2] = __hip_atomic_load(gq + 2 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    bool ready = true;
#pragma unroll
    for (int i = 0; i < 21; ++i) ready = ready && (x[i] >> 32) == 1ull;
    if (ready || it > (1 << 20)) {
#pragma unroll
      for (int qq = 0; qq < 7; ++qq) {
        ms[qq] = __uint_as_float((uint32_t)x[3 * qq]);
        ls[qq] = __uint_as_float((uint32_t)x[3 * qq + 1]);
        os[qq] = __uint_as_float((uint32_t)x[3 * qq + 2]);
      }
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int qq = 0; qq < 8; ++qq)
    if (qq == ns - 1) { ms[qq] = mm; ls[qq] = l; os[qq] = o; }
  float M = -INFINITY;
#pragma unroll
  for (int qq = 0; qq < 8; ++qq)
    if (qq < ns) M = fmaxf(M, ms[qq]);
  float lt = 0.f, ot = 0.f;
#pragma unroll
  for (int qq = 0; qq < 8; ++qq)
    if (qq < ns) {
      const float f = MODE >= 3 ? __builtin_amdgcn_exp2f(ms[qq] - M) : expf(ms[qq] - M);
      lt = fmaf(ls[qq], f, lt);
      ot = fmaf(os[qq], f, ot);
    }
  orow[tid] = f2bf(ot / lt);
#pragma unroll
  for (int qq = 0; qq < 7; ++qq)
    if (qq < ns - 1) {
      __hip_atomic_store(gr + qq * G + 2 + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid == 0) {
        __hip_atomic_store(gr + qq * G, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gr + qq * G + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
}
}  // namespace xl

extern "C" int xa_lab_attn(int mode, const void* q, const void* k, const void* v, int B, int H, int S, int ns,
                           void* gran, void* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int chunk = (S + ns - 1) / ns;
  if (chunk > 256 || chunk <= 224) return 3;
  const dim3 grid((unsigned)(B * H), (unsigned)ns);
  auto args = [&](auto ker) {
    hipLaunchKernelGGL(ker, grid, dim3(256), 0, s, (const bf16_t*)q, H, (const bf16_t*)k, (const bf16_t*)v, S, chunk,
                       (unsigned long long*)gran, (bf16_t*)out);
  };
  switch (mode) {
    case 0: args(xl::xa_kernel<0>); break;
    case 1: args(xl::xa_kernel<1>); break;
    case 2: args(xl::xa_kernel<2>); break;
    case 3: args(xl::xa_kernel<3>); break;
    case 4: args(xl::xa_kernel<4>); break;
    case 5: args(xl::xa_kernel<5>); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 4;
}
