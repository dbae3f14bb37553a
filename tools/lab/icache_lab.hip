// Instruction-fetch lab (development): is straight-line code cold at every kernel launch?
// Kernels execute the same number of VALU instructions, straight-line (.rept) or as a loop.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void straight_2000(float* out) {
  float v = threadIdx.x;
  asm volatile(".rept 2000\n\tv_add_f32 %0, 1.0, %0\n\t.endr" : "+v"(v));
  if (v == -1.f) out[0] = v;
}
__global__ void straight_500(float* out) {
  float v = threadIdx.x;
  asm volatile(".rept 500\n\tv_add_f32 %0, 1.0, %0\n\t.endr" : "+v"(v));
  if (v == -1.f) out[0] = v;
}
__global__ void loop_2000(float* out, int n) {
  float v = threadIdx.x;
  for (int i = 0; i < n; ++i) asm volatile(".rept 20\n\tv_add_f32 %0, 1.0, %0\n\t.endr" : "+v"(v));
  if (v == -1.f) out[0] = v;
}

template <typename F>
void timeit(const char* name, F launch, hipStream_t s) {
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 32; ++i) launch();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, s);
  for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s));
  hipEventRecord(e1, s); CK(hipEventSynchronize(e1));
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("%-36s : %6.2f us/launch\n", name, ms * 1000.f / 320);
}

int main() {
  hipStream_t s; CK(hipStreamCreate(&s));
  float* out; CK(hipMalloc(&out, 4096));
  for (int G : {80, 256}) {
    printf("G=%d, 256 threads\n", G);
    timeit("straight 500 v_add", [&] { hipLaunchKernelGGL(straight_500, dim3(G), dim3(256), 0, s, out); }, s);
    timeit("straight 2000 v_add", [&] { hipLaunchKernelGGL(straight_2000, dim3(G), dim3(256), 0, s, out); }, s);
    timeit("loop 100 x 20 v_add", [&] { hipLaunchKernelGGL(loop_2000, dim3(G), dim3(256), 0, s, out, 100); }, s);
    timeit("loop 25 x 20 v_add", [&] { hipLaunchKernelGGL(loop_2000, dim3(G), dim3(256), 0, s, out, 25); }, s);
  }
  return 0;
}
