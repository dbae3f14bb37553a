// Lab (not product): where the decode chain's kw_dec_linear launches spend their time, on the production geometries
// and the production launch path (kw_dec_linear over packed weights, large-v3 shapes, B = 32): o / xo (row split,
// 160 workgroups), fc1 (LayerNorm + GELU, 160), fc2 (split-K seam, 480).  declin.hip is included with its
// development hook KW_DEC_STAMP defined here: wave 0 of every workgroup stores s_memrealtime (100 MHz) at
//   0 entry | 1 its weight + activation loads landed (a vmcnt(0) is inserted there) | 2 MFMA + LayerNorm statistics
//   done | 3 reduced across waves (and, at the seam, the last arriver's partial sums loaded) | 4 epilogue stores
//   issued | 5 those stores drained (a vmcnt(0) is inserted)
// into kw_lab_stamps[workgroup][slot] (a store per stamp: lab timing, within a few percent of the product kernel).
// Each shape: 32 launches on 32 distinct weight sets captured in one hipGraph, replayed; the stamps of the LAST launch
// of the last replay are summarised (medians over workgroups, us after the first workgroup's entry).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics tools/lab/chain_stamps.hip \
//     kotoba-whisper_amd/csrc/capi.hip -o /tmp/chain_stamps && /tmp/chain_stamps
#include <hip/hip_runtime.h>
__device__ unsigned long long kw_lab_stamps[2048 * 8];
#define KW_DEC_STAMP_DECL
#define KW_DEC_STAMP(slot)                                                                                         \
  do {                                                                                                             \
    if ((slot) == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                              \
    if (threadIdx.x == 0)                                                                                          \
      kw_lab_stamps[(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + (slot)] =              \
          __builtin_amdgcn_s_memrealtime();                                                                        \
  } while (0)
#define KW_DEC_STAMP_FLUSH                                                                                         \
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                                 \
  if (threadIdx.x == 0)                                                                                            \
    kw_lab_stamps[(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + 5] = __builtin_amdgcn_s_memrealtime();
#include "../../kotoba-whisper_amd/csrc/declin.hip"

#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static double med(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

struct Shape {
  const char* name;
  int N, K, resid, ln, gelu, bf16out;
};

// fc2 geometry variants through the production kernels with a chosen Geo (ks K-splits of nw waves x ktm k-tiles)
static float fc2_geo(const char* name, int ktm, int nw, int ks, hipStream_t s, bf16_t* x, float* h, bf16_t* hb, float* bias,
                     void* ws, std::vector<void*>& Ws) {
  const int M = 32, N = 1280, K = 5120, L = (int)Ws.size();
  DecP p{};
  p.x = x; p.ldx = K; p.ln = 0; p.ln_eps = 1e-5f; p.W = nullptr; p.bias = bias; p.C = nullptr; p.ldc = N;
  p.gelu = 0; p.scale = 1.f; p.scale_cols = 0; p.h = h; p.hb = hb; p.ldh = N; p.M = M; p.N = N; p.K = K;
  p.cnt = reinterpret_cast<int*>(ws); p.slab = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + CNT_MAX * sizeof(int));
  p.xlds = 1; p.vec_epi = 1;
  Geo g{1, ktm, nw, ks};
  hipGraph_t gr; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < L; ++i) {
    p.W = reinterpret_cast<const bf16x8*>(Ws[i]);
    CK(launch(p, true, g, true, s));
  }
  CK(hipStreamEndCapture(s, &gr));
  CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-40s %6.2f us/launch\n", name, ms * 1000.f / (20 * L));
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(gr));
  return ms;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int M = 32, L = 32;
  const Shape shapes[] = {{"o / xo RESID (row split)", 1280, 1280, 1, 0, 0, 0},
                          {"fc1 LN + GELU bf16", 5120, 1280, 0, 1, 1, 1},
                          {"fc2 RESID (split-K seam)", 1280, 5120, 1, 0, 0, 0},
                          {"qkv LN (two-launch plan)", 3840, 1280, 0, 1, 0, 1}};
  bf16_t* x; CK(hipMalloc(&x, 32 * 5120 * 2)); CK(hipMemset(x, 0x3c, 32 * 5120 * 2));
  float* h; CK(hipMalloc(&h, 32 * 5120 * 4)); CK(hipMemset(h, 0, 32 * 5120 * 4));
  bf16_t* hb; CK(hipMalloc(&hb, 32 * 5120 * 2));
  void* C; CK(hipMalloc(&C, 32 * 5120 * 4));
  float* bias; CK(hipMalloc(&bias, 5120 * 4)); CK(hipMemset(bias, 0, 5120 * 4));
  float* cs; CK(hipMalloc(&cs, 5120 * 4)); CK(hipMemset(cs, 0, 5120 * 4));
  void* ws; CK(hipMalloc(&ws, 32 << 20)); CK(hipMemset(ws, 0, 32 << 20));
  std::vector<unsigned long long> st(2048 * 8);
  if (getenv("FC2_GEO")) {  // fc2 K-split geometry sweep, then exit
    std::vector<void*> Ws(L);
    for (int i = 0; i < L; ++i) { CK(hipMalloc(&Ws[i], (size_t)1280 * 5120 * 2)); CK(hipMemset(Ws[i], 0x3c, (size_t)1280 * 5120 * 2)); }
    for (int rep = 0; rep < 2; ++rep) {
      fc2_geo("fc2 ks 6 x 6 waves x 5 (product)", 5, 6, 6, s, x, h, hb, bias, ws, Ws);
      fc2_geo("fc2 ks 4 x 8 waves x 5", 5, 8, 4, s, x, h, hb, bias, ws, Ws);
      fc2_geo("fc2 ks 3 x 6 waves x 10", 10, 6, 3, s, x, h, hb, bias, ws, Ws);
      fc2_geo("fc2 ks 4 x 4 waves x 10", 10, 4, 4, s, x, h, hb, bias, ws, Ws);
      fc2_geo("fc2 ks 8 x 4 waves x 5", 5, 4, 8, s, x, h, hb, bias, ws, Ws);
      fc2_geo("fc2 ks 5 x 8 waves x 4(5)", 5, 8, 5, s, x, h, hb, bias, ws, Ws);
    }
    return 0;
  }
  for (const Shape& sh : shapes) {
    std::vector<void*> Ws(L);
    for (int i = 0; i < L; ++i) {
      CK(hipMalloc(&Ws[i], (size_t)sh.N * sh.K * 2));
      CK(hipMemset(Ws[i], 0x3c, (size_t)sh.N * sh.K * 2));
    }
    kw_dec_linear_args a{};
    a.x = x; a.ldx = sh.K; a.ln = sh.ln; a.ln_eps = 1e-5f; a.ln_colsum = cs; a.bias = bias;
    a.epilogue = sh.resid ? KW_EPI_RESID : KW_EPI_STORE;
    a.C = sh.resid ? nullptr : C; a.ldc = sh.N; a.c_dtype = sh.bf16out ? KW_DT_BF16 : KW_DT_F32;
    a.gelu = sh.gelu; a.scale = 1.f; a.scale_cols = 0;
    a.h = sh.resid ? h : nullptr; a.hb = sh.resid ? hb : nullptr; a.ldh = sh.N;
    a.M = M; a.N = sh.N; a.K = sh.K; a.workspace = ws; a.ws_bytes = 32 << 20;
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < L; ++i) {
      a.W = Ws[i];
      if (kw_dec_linear(&a, s) != 0) { printf("kw_dec_linear failed\n"); exit(1); }
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemsetAsync(ws, 0, 4096 * 4, s));  // (arrival counters are re-armed by the kernels anyway)
      unsigned long long zero[2048 * 8] = {};
      CK(hipMemcpyToSymbolAsync(HIP_SYMBOL(kw_lab_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(kw_lab_stamps), sizeof(unsigned long long) * st.size()));
      unsigned long long t0 = ~0ull, tend = 0;
      int n = 0;
      for (int w = 0; w < 2048; ++w)
        if (st[w * 8]) { t0 = std::min(t0, st[w * 8]); ++n; }
      std::vector<double> ph[6];
      int done = 0;
      for (int w = 0; w < 2048; ++w) {
        const unsigned long long* q = &st[w * 8];
        if (!q[0]) continue;
        for (int k = 0; k < 6; ++k)
          if (q[k]) ph[k].push_back((double)(q[k] - t0) / 100.0);
        if (q[5]) { tend = std::max(tend, q[5]); ++done; }
      }
      printf("%-28s %6.2f us/launch | WGs %4d (finishing %4d) | median us after first entry: entry %.2f loads %.2f mfma %.2f "
             "reduced %.2f stores-issued %.2f drained %.2f | last drained %.2f | entry spread %.2f\n",
             sh.name, ms * 1000.f / (20 * L), n, done, med(ph[0]), med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]),
             med(ph[5]), (tend - t0) / 100.0, ph[0].empty() ? 0.0 : (*std::max_element(ph[0].begin(), ph[0].end())));
    }
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    for (void* p : Ws) CK(hipFree(p));
  }
  return 0;
}
