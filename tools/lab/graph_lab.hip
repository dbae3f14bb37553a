// Lab: do two branches of one captured hipGraph run concurrently on gfx950 / ROCm 7.2?
// kernel A: publish "A started", then wait (bounded) for "B done"; kernel B: wait (bounded) for "A started",
// then publish "B done".  Both branches complete without a timeout only if they were co-resident.
// Also: hand-off latency between two kernels of the graph (one spins on the other's flag).
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ int ld_flag(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// f[0] = A started, f[1] = B done; res[0] = A's spins (-1 timeout), res[1] = B's spins, res[2..3] = clocks
__global__ void kA(int* f, long long* res, int epoch) {
  if (threadIdx.x != 0) return;
  st_flag(f + 0, epoch);
  long long t0 = wall_clock64();
  int n = 0;
  while (ld_flag(f + 1) < epoch) {
    __builtin_amdgcn_s_sleep(2);
    if (++n > (1 << 22)) { n = -1; break; }
  }
  res[0] = n;
  res[2] = wall_clock64() - t0;
}

__global__ void kB(int* f, long long* res, int epoch) {
  if (threadIdx.x != 0) return;
  long long t0 = wall_clock64();
  int n = 0;
  while (ld_flag(f + 0) < epoch) {
    __builtin_amdgcn_s_sleep(2);
    if (++n > (1 << 22)) { n = -1; break; }
  }
  st_flag(f + 1, epoch);
  res[1] = n;
  res[3] = wall_clock64() - t0;
}

extern "C" int lab_launch_a(int* f, long long* res, int epoch, void* s) {
  hipLaunchKernelGGL(kA, dim3(1), dim3(64), 0, (hipStream_t)s, f, res, epoch);
  return (int)hipGetLastError();
}
extern "C" int lab_launch_b(int* f, long long* res, int epoch, void* s) {
  hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, (hipStream_t)s, f, res, epoch);
  return (int)hipGetLastError();
}
