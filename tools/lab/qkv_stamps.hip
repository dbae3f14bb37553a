// Lab (not product): where kw_dec_qkv_self (the greedy step's fused self-attention block) spends its time, on the
// production launch path at large-v3 B = 32 (240 projection workgroups, 320 pair workgroups).  qkvself.hip is
// included with its development hooks defined here: thread 0 of every workgroup stores s_memrealtime (100 MHz) at
//   projection workgroups: 0 entry | 1 MFMAs done, partial tiles in LDS | 2 granules published
//   pair workgroups:       4 entry | 5 its q / k / v granules received (after the barrier) | 6 attention done
//                          (before the merge barrier) | 7 output stored
// into kw_lab_stamps[workgroup][slot].  32 launches on 32 layers' weights and caches captured in one hipGraph,
// replayed; the stamps of the LAST launch are summarised (medians over workgroups, us after the first entry).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics tools/lab/qkv_stamps.hip \
//     kotoba-whisper_amd/csrc/capi.hip -o /tmp/qkv_stamps && /tmp/qkv_stamps
#include <hip/hip_runtime.h>
__device__ unsigned long long kw_lab_stamps[1024 * 8];
#define KW_LAB_STAMP(slot)                                                                  \
  do {                                                                                      \
    if (threadIdx.x == 0) kw_lab_stamps[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define KW_PROJ_STAMP(slot) KW_LAB_STAMP(slot)
#define KW_QS_STAMP(slot) KW_LAB_STAMP(slot)
#include "../../kotoba-whisper_amd/csrc/qkvself.hip"

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
static double mx(const std::vector<double>& v) { return v.empty() ? 0.0 : *std::max_element(v.begin(), v.end()); }

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int M = 32, d = 1280, H = 20, T = 448, NL = 32;
  bf16_t* x; CK(hipMalloc(&x, M * d * 2)); CK(hipMemset(x, 0x3c, M * d * 2));
  float* cs; CK(hipMalloc(&cs, 3 * d * 4)); CK(hipMemset(cs, 0, 3 * d * 4));
  float* bias; CK(hipMalloc(&bias, 3 * d * 4)); CK(hipMemset(bias, 0, 3 * d * 4));
  void* out; CK(hipMalloc(&out, M * d * 2));
  const size_t wsb = kw_dec_qkv_self_workspace(M, d);
  void* ws; CK(hipMalloc(&ws, wsb)); CK(hipMemset(ws, 0, wsb));
  int32_t* cur; CK(hipMalloc(&cur, 4));
  std::vector<void*> Ws(NL), kc(NL), vc(NL);
  const size_t cache = (size_t)M * H * T * 64 * 2;
  for (int i = 0; i < NL; ++i) {
    CK(hipMalloc(&Ws[i], (size_t)3 * d * d * 2)); CK(hipMemset(Ws[i], 0x3c, (size_t)3 * d * d * 2));
    CK(hipMalloc(&kc[i], cache)); CK(hipMemset(kc[i], 0x3c, cache));
    CK(hipMalloc(&vc[i], cache)); CK(hipMemset(vc[i], 0x3c, cache));
  }
  std::vector<unsigned long long> st(1024 * 8);
  for (int L : {68, 132}) {
    CK(hipMemcpy(cur, &L, 4, hipMemcpyHostToDevice));
    kw_dec_qkv_self_args a{};
    a.x = x; a.ldx = d; a.ln_eps = 1e-5f; a.ln_colsum = cs; a.bias = bias; a.scale = 0.125f;
    a.M = M; a.d = d; a.H = H; a.t_max = T; a.cur_len = cur; a.out = out; a.workspace = ws; a.ws_bytes = wsb;
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < NL; ++i) {
      a.W = Ws[i]; a.k_cache = kc[i]; a.v_cache = vc[i];
      if (kw_dec_qkv_self(&a, s) != 0) { printf("kw_dec_qkv_self failed: %s\n", kw_last_error()); exit(1); }
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const int n_lin = 3 * d / 16;
    for (int rep = 0; rep < 3; ++rep) {
      std::vector<unsigned long long> zero(1024 * 8, 0);
      CK(hipMemcpyToSymbolAsync(HIP_SYMBOL(kw_lab_stamps), zero.data(), zero.size() * 8, 0, hipMemcpyHostToDevice, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(kw_lab_stamps), st.size() * 8));
      unsigned long long t0 = ~0ull;
      for (int w = 0; w < 1024; ++w) {
        if (st[w * 8]) t0 = std::min(t0, st[w * 8]);
        if (st[w * 8 + 4]) t0 = std::min(t0, st[w * 8 + 4]);
      }
      std::vector<double> ph[8];
      for (int w = 0; w < 1024; ++w)
        for (int k = 0; k < 8; ++k)
          if (st[w * 8 + k]) ph[k].push_back((double)(st[w * 8 + k] - t0) / 100.0);
      printf("L %3d: %6.2f us/launch | proj WGs %zu: entry %.2f (last %.2f) mfma %.2f reduced+published %.2f (last %.2f) | "
             "pair WGs %zu: entry %.2f (last %.2f) granules %.2f (last %.2f) attention %.2f out %.2f (last %.2f) | n_lin %d\n",
             L, ms * 1000.f / (20 * NL), ph[0].size(), med(ph[0]), mx(ph[0]), med(ph[1]), med(ph[2]), mx(ph[2]), ph[4].size(),
             med(ph[4]), mx(ph[4]), med(ph[5]), mx(ph[5]), med(ph[6]), med(ph[7]), mx(ph[7]), n_lin);
    }
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  }
  return 0;
}
