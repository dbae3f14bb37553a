// Workgroup -> CU placement probe (lab r05t, development tool, not part of the product).
//
// cross_attn_row_kernel's split pairs assume the dispatcher deals a grid's workgroups breadth-first over the CUs of
// each XCD (every CU's first slot, then every CU's second ...).  This launches grids with the row kernel's
// residency (256 threads, 48 KB of LDS: at most 3 workgroups per CU) and records each workgroup's hardware
// (XCC, SE, SH, CU) from s_getreg, holding every workgroup ~40 us so the whole grid is resident at once.
//
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/placement_probe tools/lab/placement_probe.hip && /tmp/placement_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <set>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256) void probe(unsigned* out, int lead) {
  extern __shared__ char lds[];
  unsigned hw = 0, xcc = 0;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  lds[threadIdx.x] = (char)hw;  // touch the LDS allocation
  const long long t0 = clock64();
  // the first `lead` workgroups leave at once (a stand-in for the fused launch's projection workgroups)
  const long long hold = (int)blockIdx.x < lead ? 2000 : 100000;
  while (clock64() - t0 < hold) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = hw;
    out[3 * blockIdx.x + 1] = xcc;
    out[3 * blockIdx.x + 2] = (unsigned)lds[1];
  }
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grids[][2] = {{640, 0}, {768, 0}, {720, 80}, {848, 80}, {500, 0}};
  unsigned* d = nullptr;
  hipMalloc(&d, 3 * 1024 * sizeof(unsigned));
  int per = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&probe), 256, 48 * 1024);
  printf("{\"cus\": %d, \"blocks_per_cu\": %d}\n", ncu, per);
  for (auto& g : grids) {
    const int n = g[0], lead = g[1];
    hipLaunchKernelGGL(probe, dim3(n), dim3(256), 48 * 1024, 0, d, lead);
    std::vector<unsigned> h(3 * n);
    hipMemcpy(h.data(), d, 3 * n * sizeof(unsigned), hipMemcpyDeviceToHost);
    // CU key: (xcc, se, sh, cu) from HW_ID (gfx9 layout: cu 11:8, sh 12, se 15:13)
    std::map<std::tuple<unsigned, unsigned, unsigned, unsigned>, std::vector<int>> cu;
    for (int b = 0; b < n; ++b) {
      const unsigned hw = h[3 * b], x = h[3 * b + 1] & 0xf;
      cu[{x, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15}].push_back(b);
    }
    // per CU: how many of its workgroups fall in each third of the pair range [lead, n)
    std::map<std::vector<int>, int> hist;  // (count in [lead, lead+2C), count in [lead+2C, n), leads) -> CUs
    int maxw = 0;
    for (auto& kv : cu) {
      int a = 0, c = 0, l = 0;
      for (int b : kv.second) {
        if (b < lead) ++l;
        else if (b < lead + 2 * ncu) ++a;
        else ++c;
      }
      hist[{a, c, l}]++;
      if ((int)kv.second.size() > maxw) maxw = kv.second.size();
    }
    printf("{\"grid\": %d, \"lead\": %d, \"cus_used\": %zu, \"max_wg_per_cu\": %d, \"per_cu [first 2C, rest, lead] -> CUs\": {",
           n, lead, cu.size(), maxw);
    bool first = true;
    for (auto& kv : hist) {
      printf("%s\"%d,%d,%d\": %d", first ? "" : ", ", kv.first[0], kv.first[1], kv.first[2], kv.second);
      first = false;
    }
    printf("}}\n");
  }
  hipFree(d);
  return 0;
}
