// Lab: the production dec_linear kernel (declin.hip, included) vs stripped variants, same geometry.
#include <hip/hip_runtime.h>
// stamps kept in registers, written at the end into p.slab + 4 MB (the slab is unused at KS = 1);
// slot 1 waits for the wave's loads (vmcnt(0)) so it reads "landed"
#define KW_DEC_STAMP_DECL unsigned long long kw_st_[5] = {0, 0, 0, 0, 0};
#define KW_DEC_STAMP(slot)                                                                         \
  do {                                                                                             \
    if ((slot) == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                              \
    kw_st_[slot] = __builtin_amdgcn_s_memrealtime();                                               \
  } while (0)
#define KW_DEC_STAMP_FLUSH                                                                         \
  if (threadIdx.x == 0 && ksn == 1) {                                                              \
    unsigned long long* q_ = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(p.slab) + (4 << 20)) + blockIdx.x * 8; \
    for (int k_ = 0; k_ < 5; ++k_) q_[k_] = kw_st_[k_];                                            \
  }
#include "../../kotoba-whisper_amd/csrc/declin.hip"

#include <stdio.h>
#include <vector>
#include <algorithm>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
int kw_set_error(hipError_t) { return 2; }
int kw_set_error_msg(int c, const char*) { return c; }

template <int KTM, int NCB, bool LNA, int EPI, typename TC>
float run(const char* name, DecP p, int nw, int ks, std::vector<const bf16x8*>& Ws, hipStream_t s) {
  dim3 grid((p.N + 16 * NCB - 1) / (16 * NCB), ks), block(64 * nw);
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  p.xlds = ks == 1 && (int)grid.x <= 256;
  const size_t shm = x_lds_bytes_for(p.K / 32, p.xlds);
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&dec_linear_kernel<KTM, NCB, LNA, EPI, TC>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  for (auto* W : Ws) { p.W = W; hipLaunchKernelGGL((dec_linear_kernel<KTM, NCB, LNA, EPI, TC>), grid, block, shm, s, p, ks); }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, s);
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
  hipEventRecord(e1, s); CK(hipEventSynchronize(e1));
  float ms; hipEventElapsedTime(&ms, e0, e1);
  float us = ms * 1000.f / (20 * Ws.size());
  printf("%-40s N=%5d K=%5d : %7.2f us\n", name, p.N, p.K, us);
  if (getenv("STAMPS") && ks == 1) {
    std::vector<unsigned long long> h(1024 * 8);
    CK(hipMemcpy(h.data(), reinterpret_cast<char*>(p.slab) + (4 << 20), h.size() * 8, hipMemcpyDeviceToHost));
    double d[5] = {0}; int n = 0;
    unsigned long long t0 = ~0ull, te = 0;
    for (int b = 0; b < (int)grid.x; ++b) {
      const unsigned long long* q = &h[b * 8];
      if (!q[0]) continue;
      ++n; t0 = std::min(t0, q[0]); te = std::max(te, q[4]);
      for (int k = 1; k < 5; ++k) d[k] += (double)(q[k] - q[0]) / 100.0;
    }
    printf("   stamps (wave 0 of each WG, from its entry): loads landed %.2f | mfma %.2f | reduced %.2f | end %.2f | first entry -> last end %.2f us\n",
           d[1] / n, d[2] / n, d[3] / n, d[4] / n, (te - t0) / 100.0);
  }
  return us;
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;
}
__global__ void touch_kernel(const float* __restrict__ x, float* __restrict__ y) {
  // one dependent global round trip + store per lane
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  y[i] = x[i] + 1.f;
}
static void floor_runs(hipStream_t s) {
  float* x; CK(hipMalloc(&x, 1 << 22)); CK(hipMemset(x, 0, 1 << 22));
  for (int kind = 0; kind < 4; ++kind) {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 32; ++i) {
      if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
      if (kind == 1) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, nullptr);
      if (kind == 2) hipLaunchKernelGGL(touch_kernel, dim3(80), dim3(256), 0, s, x + (i & 1) * 65536, x + ((i + 1) & 1) * 65536);
      if (kind == 3) hipLaunchKernelGGL(touch_kernel, dim3(1024), dim3(256), 0, s, x + (i & 1) * 262144, x + ((i + 1) & 1) * 262144);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0, s);
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
    hipEventRecord(e1, s); CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const char* nm[] = {"empty 1 WG", "empty 256 WGs", "touch 80 WGs (dependent chain)", "touch 1024 WGs (dependent chain)"};
    printf("%-40s : %7.2f us per launch\n", nm[kind], ms * 1000.f / (20 * 32));
  }
}

int main() {
  hipStream_t s; CK(hipStreamCreate(&s));
  floor_runs(s);
  const int L = 32;
  bf16_t* x; CK(hipMalloc(&x, 32 * 5120 * 2)); CK(hipMemset(x, 0x3c, 32 * 5120 * 2));
  float* out; CK(hipMalloc(&out, 32 * 5120 * 4 * 2));
  float* h; CK(hipMalloc(&h, 32 * 5120 * 4));
  bf16_t* hb; CK(hipMalloc(&hb, 32 * 5120 * 2));
  float* bias; CK(hipMalloc(&bias, 5120 * 4)); CK(hipMemset(bias, 0, 5120 * 4));
  float* cs; CK(hipMalloc(&cs, 5120 * 4)); CK(hipMemset(cs, 0, 5120 * 4));
  void* ws; CK(hipMalloc(&ws, 16 << 20)); CK(hipMemset(ws, 0, 16 << 20));
  std::vector<const bf16x8*> W1(L), W3(L), W5(L), W5k(L);
  for (int i = 0; i < L; ++i) {
    bf16x8* p;
    CK(hipMalloc(&p, 3840 * 1280 * 2)); CK(hipMemset(p, 0x3c, 3840 * 1280 * 2)); W3[i] = p;
    CK(hipMalloc(&p, 1280 * 1280 * 2)); CK(hipMemset(p, 0x3c, 1280 * 1280 * 2)); W1[i] = p;
    CK(hipMalloc(&p, 5120 * 1280 * 2)); CK(hipMemset(p, 0x3c, 5120 * 1280 * 2)); W5[i] = p;
    CK(hipMalloc(&p, 5120 * 1280 * 2)); CK(hipMemset(p, 0x3c, 5120 * 1280 * 2)); W5k[i] = p;
  }
  DecP p{};
  p.x = x; p.ldx = 1280; p.ln = 0; p.ln_eps = 1e-5f; p.ln_colsum = cs; p.bias = nullptr;
  p.C = out; p.ldc = 3840; p.gelu = 0; p.scale = 1.f; p.scale_cols = 0; p.h = h; p.hb = hb; p.ldh = 1280;
  p.M = 32; p.K = 1280; p.cnt = (int*)ws; p.slab = (float*)((char*)ws + 4096 * 4);
  // qkv geometry: KTM 5, NCB 1, 8 waves
  p.N = 3840;
  run<5, 1, false, KW_EPI_STORE, float>("qkv plain f32 out", p, 8, 1, W3, s);
  run<5, 1, false, KW_EPI_STORE, bf16_t>("qkv plain bf16 out", p, 8, 1, W3, s);
  p.bias = bias;
  run<5, 1, false, KW_EPI_STORE, bf16_t>("qkv +bias bf16", p, 8, 1, W3, s);
  p.scale = 0.125f; p.scale_cols = 1280;
  run<5, 1, false, KW_EPI_STORE, bf16_t>("qkv +bias+scale bf16", p, 8, 1, W3, s);
  run<5, 1, true, KW_EPI_STORE, bf16_t>("qkv +LN+bias+scale bf16 (prod)", p, 8, 1, W3, s);
  p.scale = 1.f; p.scale_cols = 0; p.bias = nullptr;
  // o geometry: KTM 10, NCB 1, 4 waves
  p.N = 1280; p.ldc = 1280;
  run<10, 1, false, KW_EPI_STORE, float>("o plain f32", p, 4, 1, W1, s);
  p.bias = bias;
  run<10, 1, false, KW_EPI_RESID, float>("o RESID (prod)", p, 4, 1, W1, s);
  run<10, 1, true, KW_EPI_STORE, bf16_t>("xq LN (prod-like)", p, 4, 1, W1, s);
  // fc1: KTM 10, NCB 2, 4 waves
  p.N = 5120; p.ldc = 5120; p.bias = nullptr;
  run<10, 2, false, KW_EPI_STORE, float>("fc1 plain f32", p, 4, 1, W5, s);
  p.bias = bias; p.gelu = 1;
  run<10, 2, false, KW_EPI_STORE, bf16_t>("fc1 +bias+gelu bf16", p, 4, 1, W5, s);
  run<10, 2, true, KW_EPI_STORE, bf16_t>("fc1 +LN+bias+gelu bf16 (prod)", p, 4, 1, W5, s);
  p.gelu = 0;
  // fc2: K 5120, KTM 10, NCB 1, 2 waves, KS 8
  p.N = 1280; p.K = 5120; p.ldx = 5120; p.ldc = 1280; p.bias = nullptr;
  run<10, 1, false, KW_EPI_STORE, float>("fc2 plain f32 KS8", p, 2, 8, W5k, s);
  p.bias = bias;
  run<10, 1, false, KW_EPI_RESID, float>("fc2 RESID KS8 (prod)", p, 2, 8, W5k, s);
  run<5, 1, false, KW_EPI_RESID, float>("fc2 RESID 4w KTM5 KS8", p, 4, 8, W5k, s);
  // the same launches with one weight set repeated: weights L2/MALL-resident (what a prefetch buys)
  std::vector<const bf16x8*> H1(L, W1[0]), H5(L, W5[0]), H5k(L, W5k[0]);
  run<10, 1, false, KW_EPI_RESID, float>("fc2 RESID KS8 (prod) HOT", p, 2, 8, H5k, s);
  p.N = 1280; p.K = 1280; p.ldx = 1280; p.ldc = 1280;
  run<10, 1, false, KW_EPI_RESID, float>("o RESID (prod) HOT", p, 4, 1, H1, s);
  run<10, 1, true, KW_EPI_STORE, bf16_t>("xq LN (prod-like) HOT", p, 4, 1, H1, s);
  p.N = 5120; p.ldc = 5120; p.gelu = 1;
  run<10, 2, true, KW_EPI_STORE, bf16_t>("fc1 +LN+bias+gelu bf16 (prod) HOT", p, 4, 1, H5, s);
  // empty-ish: K = 64 (one k-tile), launch + chain floor
  p.gelu = 0; p.N = 1280; p.K = 64; p.ldx = 64; p.ldc = 1280;
  run<10, 1, false, KW_EPI_RESID, float>("floor: o-geometry K=64 HOT", p, 4, 1, H1, s);
  return 0;
}
