// GEMM timeline lab (development): builds gemm.hip with s_memrealtime stamps at the tile-loop points
// (KW_GEMM_STAMP) and prints, over all workgroups, the time to the first main loop, per-tile main
// loop / epilogue / hand-off spans.  bash tools/lab/dbg.sh-style: hipcc, run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

__device__ unsigned long long* g_stamps;
#define KW_GEMM_STAMP(slot)                                                                     \
  do {                                                                                          \
    if (threadIdx.x == 0 && (slot) < 64) g_stamps[blockIdx.x * 64 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#include "../../kotoba-whisper_amd/csrc/gemm.hip"

static void fill(unsigned short* d, size_t n, unsigned seed) {
  std::vector<unsigned short> h(n);
  unsigned s = seed;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    float f = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
    unsigned u;
    memcpy(&u, &f, 4);
    h[i] = (unsigned short)(u >> 16);
  }
  hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 48000, N = argc > 2 ? atoi(argv[2]) : 1280, K = argc > 3 ? atoi(argv[3]) : 1280;
  const int mode = argc > 4 ? atoi(argv[4]) : 0;  // 0 store bf16, 1 bias+GELU bf16, 2 residual add into f32, 3 bias + store bf16
  unsigned short *A, *W, *C;
  float* bias;
  hipMalloc(&A, (size_t)M * K * 2);
  hipMalloc(&W, (size_t)N * K * 2);
  hipMalloc(&C, (size_t)M * N * 4);
  hipMalloc(&bias, (size_t)N * 4);
  hipMemset(bias, 0, (size_t)N * 4);
  hipMemset(C, 0, (size_t)M * N * 4);
  fill(A, (size_t)M * K, 1);
  fill(W, (size_t)N * K, 2);
  unsigned long long* st;
  const int G = 256;
  hipMalloc(&st, G * 64 * 8);
  hipMemset(st, 0, G * 64 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st));
  kw_gemm_args a = {};
  a.dtype = KW_DT_BF16; a.c_dtype = KW_DT_BF16; a.A = A; a.lda = K; a.W = W; a.C = C; a.ldc = N;
  a.M = M; a.N = N; a.K = K; a.epilogue = KW_EPI_STORE; a.scale = 1.f;
  if (mode == 1) { a.gelu = 1; a.bias = bias; }
  if (mode == 3) a.bias = bias;  // bias, no GELU
  if (mode == 2) { a.epilogue = KW_EPI_RESID; a.c_dtype = KW_DT_F32; a.bias = bias; }
  for (int i = 0; i < 20; ++i) kw_gemm(&a, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  kw_gemm(&a, 0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(G * 64);
  hipMemcpy(h.data(), st, G * 64 * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, tend = 0;
  for (int b = 0; b < G; ++b) if (h[b * 64]) t0 = std::min(t0, h[b * 64]);
  // per tile slots: 1+3t main start, 2+3t main end, 3+3t epilogue end
  double s_start = 0, s_main = 0, s_epi = 0, s_gap = 0;
  int n_main = 0, n_gap = 0, n_wg = 0;
  double first_main_max = 0, start_max = 0;
  for (int b = 0; b < G; ++b) {
    if (!h[b * 64]) continue;
    ++n_wg;
    start_max = std::max(start_max, (h[b * 64] - t0) / 100.0);
    s_start += (h[b * 64 + 1] - h[b * 64]) / 100.0;
    first_main_max = std::max(first_main_max, (h[b * 64 + 1] - t0) / 100.0);
    for (int t = 0; t < 20; ++t) {
      const unsigned long long a1 = h[b * 64 + 1 + 3 * t], a2 = h[b * 64 + 2 + 3 * t], a3 = h[b * 64 + 3 + 3 * t];
      if (!a1 || !a2 || !a3) break;
      s_main += (a2 - a1) / 100.0; s_epi += (a3 - a2) / 100.0; ++n_main;
      tend = std::max(tend, a3);
      const unsigned long long nx = h[b * 64 + 1 + 3 * (t + 1)];
      if (t + 1 < 20 && nx) { s_gap += (nx - a3) / 100.0; ++n_gap; }
    }
  }
  printf("mode %d ", mode);
  printf("M=%d N=%d K=%d  event %.1f us  stamped span %.1f us  WGs %d  last WG start %.2f us  first-main max %.2f us\n",
         M, N, K, ms * 1e3, (tend - t0) / 100.0, n_wg, start_max, first_main_max);
  printf("avg: entry->main %.2f us | main loop %.2f us | epilogue %.2f us | epilogue->next main %.2f us | tiles %d\n",
         s_start / n_wg, s_main / n_main, s_epi / n_main, n_gap ? s_gap / n_gap : 0.0, n_main);
  for (int b = 0; b < 3; ++b) {
    printf("wg %d:", b);
    for (int sl = 0; sl < 16 && h[b * 64 + sl]; ++sl) printf(" %.2f", (h[b * 64 + sl] - t0) / 100.0);
    printf("\n");
  }
  return 0;
}
