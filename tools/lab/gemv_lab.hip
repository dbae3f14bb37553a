// Decode GEMV design lab (development tool, not product code): M = 32 rows, bf16 x in L2, weights packed
// as 1-KB 16x32 MFMA B-fragments [N/16][K/32][64][8].  Times 32 launches (32 distinct weight buffers,
// as 32 decoder layers) captured in a hipGraph; prints us per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void empty_kernel(float* p) { if (threadIdx.x == 9999) p[0] = 1.f; }

// WPB waves per WG; the WG owns 16 columns and a K-range of KT*WPB k-tiles (KS WGs split K; atomicAdd f32)
template <int WPB, int KT, int KS>
__global__ __launch_bounds__(WPB * 64) void gemv_v1(const bf16x8* __restrict__ W, const __bf16* __restrict__ x,
                                                    float* __restrict__ out, int N, int K) {
  __shared__ f32x4 red[WPB][2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = blockIdx.x, ks = blockIdx.y;
  const int nkt = K >> 5;
  const int kt0 = (ks * WPB + wave) * KT;
  const bf16x8* wp = W + ((long)cb * nkt + kt0) * 64 + lane;
  const int arow = lane & 15, akoff = 8 * (lane >> 4);
  bf16x8 w[KT], a0[KT], a1[KT];
#pragma unroll
  for (int u = 0; u < KT; ++u) w[u] = __builtin_nontemporal_load(wp + u * 64);
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    const int k = (kt0 + u) * 32 + akoff;
    a0[u] = *reinterpret_cast<const bf16x8*>(x + (long)arow * K + k);
    a1[u] = *reinterpret_cast<const bf16x8*>(x + (long)(16 + arow) * K + k);
  }
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0;
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], w[u], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], w[u], c1, 0, 0, 0);
  }
  if (WPB > 1) {
    red[wave][0][lane] = c0;
    red[wave][1][lane] = c1;
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int w2 = 1; w2 < WPB; ++w2) {
      c0 += red[w2][0][lane];
      c1 += red[w2][1][lane];
    }
  }
  const int col = cb * 16 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m0 = 4 * (lane >> 4) + r;
    if (KS == 1) {
      out[(long)m0 * N + col] = c0[r];
      out[(long)(16 + m0) * N + col] = c1[r];
    } else {
      atomicAdd(out + (long)m0 * N + col, c0[r]);
      atomicAdd(out + (long)(16 + m0) * N + col, c1[r]);
    }
  }
}

template <int WPB, int KT, int KS>
float run(const char* name, int N, int K, std::vector<bf16x8*>& Ws, __bf16* x, float* out, hipStream_t s) {
  const int nkt = K / 32;
  if (nkt != WPB * KT * KS) { printf("%s: bad config\n", name); return 0; }
  dim3 grid(N / 16, KS);
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (auto* W : Ws) hipLaunchKernelGGL((gemv_v1<WPB, KT, KS>), grid, dim3(WPB * 64), 0, s, W, x, out, N, K);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, s);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  hipEventRecord(e1, s);
  CK(hipEventSynchronize(e1));
  float ms; hipEventElapsedTime(&ms, e0, e1);
  float us = ms * 1000.f / (reps * Ws.size());
  printf("%-28s N=%5d K=%5d WGs=%5d thr=%4d : %7.2f us  %6.0f GB/s\n", name, N, K, N / 16 * KS, WPB * 64, us,
         (double)N * K * 2 / us / 1e3);
  hipGraphExecDestroy(ge); hipGraphDestroy(g);
  return us;
}


// v2: each wave owns NCB column blocks (x fragments reused NCB times) and KT k-tiles; WPB waves split the
// WG's K-range; KS workgroups split K with a deterministic seam (SEAM=1: sc1 slab + arrival counter, the
// last arriver sums the KS partials in fixed order) or none (KS == 1).  LNTAIL=1: after its column block
// completes, a WG bumps a global counter and the grid's last WG re-reads all 32 x N outputs (sc1) and
// writes a normalised bf16 copy (the LayerNorm-in-producer tail).
template <int WPB, int KT, int NCB, int KS, int LNTAIL>
__global__ __launch_bounds__(WPB * 64) void gemv_v2(const bf16x8* __restrict__ W, const __bf16* __restrict__ x,
                                                    float* __restrict__ out, int N, int K, float* __restrict__ slab,
                                                    int* __restrict__ cnt, __bf16* __restrict__ xo) {
  __shared__ f32x4 red[WPB][NCB][2][64];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = blockIdx.x, ks = blockIdx.y;  // column group of NCB blocks
  const int nkt = K >> 5;
  const int kt0 = (ks * WPB + wave) * KT;
  const int arow = lane & 15, akoff = 8 * (lane >> 4);
  bf16x8 w[NCB][KT], a0[KT], a1[KT];
#pragma unroll
  for (int c = 0; c < NCB; ++c)
#pragma unroll
    for (int u = 0; u < KT; ++u) w[c][u] = __builtin_nontemporal_load(W + ((long)(cg * NCB + c) * nkt + kt0 + u) * 64 + lane);
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    const int k = (kt0 + u) * 32 + akoff;
    a0[u] = *reinterpret_cast<const bf16x8*>(x + (long)arow * K + k);
    a1[u] = *reinterpret_cast<const bf16x8*>(x + (long)(16 + arow) * K + k);
  }
  f32x4 c0[NCB], c1[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) { c0[c] = f32x4{0, 0, 0, 0}; c1[c] = c0[c]; }
#pragma unroll
  for (int u = 0; u < KT; ++u)
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      c0[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], w[c][u], c0[c], 0, 0, 0);
      c1[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], w[c][u], c1[c], 0, 0, 0);
    }
  if (WPB > 1) {
#pragma unroll
    for (int c = 0; c < NCB; ++c) { red[wave][c][0][lane] = c0[c]; red[wave][c][1][lane] = c1[c]; }
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int w2 = 1; w2 < WPB; ++w2)
#pragma unroll
      for (int c = 0; c < NCB; ++c) { c0[c] += red[w2][c][0][lane]; c1[c] += red[w2][c][1][lane]; }
  }
  // (only wave 0 continues when WPB > 1)
  if (KS > 1) {
    float* sl = slab + ((long)cg * KS + ks) * (NCB * 512);
#pragma unroll
    for (int c = 0; c < NCB; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        __hip_atomic_store(sl + c * 512 + r * 64 + lane, c0[c][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sl + c * 512 + 256 + r * 64 + lane, c1[c][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) {
      const int prev = __hip_atomic_fetch_add(cnt + cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == KS - 1;
      if (last) __hip_atomic_store(cnt + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = __shfl(last, 0, 64);
    if (!last) return;
    const float* s0 = slab + (long)cg * KS * (NCB * 512);
#pragma unroll
    for (int c = 0; c < NCB; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = 0.f, v1 = 0.f;
        for (int q = 0; q < KS; ++q) {
          v0 += __hip_atomic_load(s0 + q * NCB * 512 + c * 512 + r * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v1 += __hip_atomic_load(s0 + q * NCB * 512 + c * 512 + 256 + r * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        c0[c][r] = v0;
        c1[c][r] = v1;
      }
  }
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int col = (cg * NCB + c) * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m0 = 4 * (lane >> 4) + r;
      if (LNTAIL) {
        __hip_atomic_store(out + (long)m0 * N + col, c0[c][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(out + (long)(16 + m0) * N + col, c1[c][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        out[(long)m0 * N + col] = c0[c][r];
        out[(long)(16 + m0) * N + col] = c1[c][r];
      }
    }
  }
  if (LNTAIL) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    const int ng = gridDim.x;
    if (lane == 0) {
      const int prev = __hip_atomic_fetch_add(cnt + 4095, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == ng - 1;
      if (last) __hip_atomic_store(cnt + 4095, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = __shfl(last, 0, 64);
    if (!last) return;
    // one wave normalises 32 rows x N (sc1 loads, 4 floats per lane per step)
    for (int m = 0; m < 32; ++m) {
      float s = 0.f, s2 = 0.f;
      for (int n = lane * 4; n < N; n += 256) {
        for (int e = 0; e < 4; ++e) {
          const float v = __hip_atomic_load(out + (long)m * N + n + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s += v; s2 += v * v;
        }
      }
      for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); s2 += __shfl_xor(s2, o, 64); }
      const float mean = s / N, rstd = rsqrtf(fmaxf(s2 / N - mean * mean, 0.f) + 1e-5f);
      for (int n = lane * 4; n < N; n += 256)
        for (int e = 0; e < 4; ++e)
          xo[(long)m * N + n + e] = (__bf16)((__hip_atomic_load(out + (long)m * N + n + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - mean) * rstd);
    }
  }
}

float* g_slab; int* g_cnt; __bf16* g_xo;

template <int WPB, int KT, int NCB, int KS, int LNTAIL>
float run2(const char* name, int N, int K, std::vector<bf16x8*>& Ws, __bf16* x, float* out, hipStream_t s) {
  const int nkt = K / 32;
  if (nkt != WPB * KT * KS || (N / 16) % NCB) { printf("%s: bad config\n", name); return 0; }
  dim3 grid(N / 16 / NCB, KS);
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (auto* W : Ws) hipLaunchKernelGGL((gemv_v2<WPB, KT, NCB, KS, LNTAIL>), grid, dim3(WPB * 64), 0, s, W, x, out, N, K, g_slab, g_cnt, g_xo);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, s);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  hipEventRecord(e1, s);
  CK(hipEventSynchronize(e1));
  float ms; hipEventElapsedTime(&ms, e0, e1);
  float us = ms * 1000.f / (reps * Ws.size());
  printf("%-34s N=%5d K=%5d WGs=%5d thr=%4d : %7.2f us  %6.0f GB/s\n", name, N, K, N / 16 / NCB * KS, WPB * 64, us,
         (double)N * K * 2 / us / 1e3);
  hipGraphExecDestroy(ge); hipGraphDestroy(g);
  return us;
}

int main() {
  hipStream_t s; CK(hipStreamCreate(&s));
  const int L = 32;
  __bf16* x; CK(hipMalloc(&x, 32 * 5120 * 2)); CK(hipMemset(x, 0, 32 * 5120 * 2));
  float* out; CK(hipMalloc(&out, 32 * 51872 * 4));
  std::vector<bf16x8*> W1(L), W3(L), W5(L), W5k(L);
  for (int i = 0; i < L; ++i) {
    CK(hipMalloc(&W1[i], 1280 * 1280 * 2)); CK(hipMemset(W1[i], 0, 1280 * 1280 * 2));
    CK(hipMalloc(&W3[i], 3840 * 1280 * 2)); CK(hipMemset(W3[i], 0, 3840 * 1280 * 2));
    CK(hipMalloc(&W5[i], 5120 * 1280 * 2)); CK(hipMemset(W5[i], 0, 5120 * 1280 * 2));
    CK(hipMalloc(&W5k[i], 1280 * 5120 * 2)); CK(hipMemset(W5k[i], 0, 1280 * 5120 * 2));
  }
  {  // empty kernel boundary
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < L; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, out);
    CK(hipStreamEndCapture(s, &g)); CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0, s);
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
    hipEventRecord(e1, s); CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("empty kernel (256 WG) in graph: %.2f us per launch\n", ms * 1000.f / (20 * L));
  }
  // N=1280, K=1280 (40 k-tiles)
  run<1, 40, 1>("o: 1 wave x 40kt", 1280, 1280, W1, x, out, s);
  run<4, 10, 1>("o: 4 waves x 10kt", 1280, 1280, W1, x, out, s);
  run<8, 5, 1>("o: 8 waves x 5kt", 1280, 1280, W1, x, out, s);
  run<4, 5, 2>("o: 4w x 5kt x KS2 atomic", 1280, 1280, W1, x, out, s);
  run<4, 2, 5>("o: 4w x 2kt x KS5 atomic", 1280, 1280, W1, x, out, s);
  run<2, 5, 4>("o: 2w x 5kt x KS4 atomic", 1280, 1280, W1, x, out, s);
  run<1, 10, 4>("o: 1w x 10kt x KS4 atomic", 1280, 1280, W1, x, out, s);
  run<1, 5, 8>("o: 1w x 5kt x KS8 atomic", 1280, 1280, W1, x, out, s);
  // N=3840
  run<4, 10, 1>("qkv: 4 waves x 10kt", 3840, 1280, W3, x, out, s);
  run<8, 5, 1>("qkv: 8 waves x 5kt", 3840, 1280, W3, x, out, s);
  run<2, 10, 2>("qkv: 2w x 10kt x KS2", 3840, 1280, W3, x, out, s);
  run<1, 10, 4>("qkv: 1w x 10kt x KS4", 3840, 1280, W3, x, out, s);
  // N=5120
  run<4, 10, 1>("fc1: 4 waves x 10kt", 5120, 1280, W5, x, out, s);
  run<8, 5, 1>("fc1: 8 waves x 5kt", 5120, 1280, W5, x, out, s);
  run<1, 10, 4>("fc1: 1w x 10kt x KS4", 5120, 1280, W5, x, out, s);
  run<2, 10, 2>("fc1: 2w x 10kt x KS2", 5120, 1280, W5, x, out, s);
  // N=1280, K=5120 (160 k-tiles)
  run<16, 10, 1>("fc2: 16 waves x 10kt", 1280, 5120, W5k, x, out, s);
  run<8, 10, 2>("fc2: 8w x 10kt x KS2", 1280, 5120, W5k, x, out, s);
  run<4, 10, 4>("fc2: 4w x 10kt x KS4", 1280, 5120, W5k, x, out, s);
  run<4, 5, 8>("fc2: 4w x 5kt x KS8", 1280, 5120, W5k, x, out, s);
  run<2, 10, 8>("fc2: 2w x 10kt x KS8", 1280, 5120, W5k, x, out, s);
  run<1, 10, 16>("fc2: 1w x 10kt x KS16", 1280, 5120, W5k, x, out, s);
  // LM head N=51872 (one buffer)
  std::vector<bf16x8*> Wl(1);
  CK(hipMalloc(&Wl[0], (size_t)51872 * 1280 * 2)); CK(hipMemset(Wl[0], 0, (size_t)51872 * 1280 * 2));
  run<4, 10, 1>("lm: 4 waves x 10kt", 51872, 1280, Wl, x, out, s);
  run<8, 5, 1>("lm: 8 waves x 5kt", 51872, 1280, Wl, x, out, s);
  run<2, 20, 1>("lm: 2 waves x 20kt", 51872, 1280, Wl, x, out, s);
  run<1, 40, 1>("lm: 1 wave x 40kt", 51872, 1280, Wl, x, out, s);
  CK(hipMalloc(&g_slab, 64 << 20)); CK(hipMalloc(&g_cnt, 4096 * 4)); CK(hipMemset(g_cnt, 0, 4096 * 4));
  CK(hipMalloc(&g_xo, 32 * 51872 * 2));
  printf("--- v2: x reuse (NCB), deterministic seam (KS), LN tail\n");
  run2<4, 10, 1, 1, 0>("o: v2 4w 10kt", 1280, 1280, W1, x, out, s);
  run2<4, 5, 1, 2, 0>("o: v2 4w 5kt KS2 seam", 1280, 1280, W1, x, out, s);
  run2<4, 2, 1, 5, 0>("o: v2 4w 2kt KS5 seam", 1280, 1280, W1, x, out, s);
  run2<1, 10, 1, 4, 0>("o: v2 1w 10kt KS4 seam", 1280, 1280, W1, x, out, s);
  run2<1, 5, 1, 8, 0>("o: v2 1w 5kt KS8 seam", 1280, 1280, W1, x, out, s);
  run2<2, 5, 1, 4, 0>("o: v2 2w 5kt KS4 seam", 1280, 1280, W1, x, out, s);
  run2<2, 5, 1, 4, 1>("o: v2 2w 5kt KS4 seam + LN tail", 1280, 1280, W1, x, out, s);
  run2<4, 10, 1, 1, 1>("o: v2 4w 10kt + LN tail", 1280, 1280, W1, x, out, s);
  run2<4, 10, 2, 1, 0>("qkv: v2 4w 10kt NCB2", 3840, 1280, W3, x, out, s);
  run2<8, 5, 2, 1, 0>("qkv: v2 8w 5kt NCB2", 3840, 1280, W3, x, out, s);
  run2<2, 10, 1, 2, 0>("qkv: v2 2w 10kt KS2 seam", 3840, 1280, W3, x, out, s);
  run2<4, 5, 2, 2, 0>("qkv: v2 4w 5kt NCB2 KS2 seam", 3840, 1280, W3, x, out, s);
  run2<4, 10, 2, 1, 0>("fc1: v2 4w 10kt NCB2", 5120, 1280, W5, x, out, s);
  run2<4, 5, 2, 2, 0>("fc1: v2 4w 5kt NCB2 KS2 seam", 5120, 1280, W5, x, out, s);
  run2<2, 10, 1, 2, 0>("fc1: v2 2w 10kt KS2 seam", 5120, 1280, W5, x, out, s);
  run2<1, 10, 1, 4, 0>("fc1: v2 1w 10kt KS4 seam", 5120, 1280, W5, x, out, s);
  run2<4, 10, 1, 4, 0>("fc2: v2 4w 10kt KS4 seam", 1280, 5120, W5k, x, out, s);
  run2<4, 5, 1, 8, 0>("fc2: v2 4w 5kt KS8 seam", 1280, 5120, W5k, x, out, s);
  run2<2, 10, 1, 8, 0>("fc2: v2 2w 10kt KS8 seam", 1280, 5120, W5k, x, out, s);
  run2<1, 10, 1, 16, 0>("fc2: v2 1w 10kt KS16 seam", 1280, 5120, W5k, x, out, s);
  run2<2, 10, 1, 8, 1>("fc2: v2 2w 10kt KS8 seam + LN tail", 1280, 5120, W5k, x, out, s);
  run2<4, 10, 2, 1, 0>("lm: v2 4w 10kt NCB2", 51872, 1280, Wl, x, out, s);
  run2<4, 10, 4, 1, 0>("lm: v2 4w 10kt NCB4", 51872, 1280, Wl, x, out, s);
  run2<8, 5, 4, 1, 0>("lm: v2 8w 5kt NCB4", 51872, 1280, Wl, x, out, s);
  run2<2, 10, 2, 2, 0>("lm: v2 2w 10kt NCB2 KS2 seam", 51872, 1280, Wl, x, out, s);
  run2<4, 5, 4, 2, 0>("lm: v2 4w 5kt NCB4 KS2 seam", 51872, 1280, Wl, x, out, s);
  return 0;
}
