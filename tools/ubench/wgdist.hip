// wgdist.hip -- how does the dispatcher place the hot kernel's grid on CUs?
// k_sha1_fixed at 131072 chunks is 512 workgroups x 256 threads with 110
// VGPRs (occupancy limit 4 waves/SIMD = 4 workgroups per CU), i.e. 2 per CU on
// average.  This probe launches the same shape (same VGPR allocation, long-running
// waves so the whole grid is co-resident) and records each wave's hardware
// location, then histograms workgroups per CU.  With dynamic LDS per workgroup
// > 160 KiB / 3 the hardware cannot place a third workgroup on a CU.
// Args: none.  Prints the histogram for LDS pads 0 and 56 KiB.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_probe(uint32_t *rec, uint64_t spin_cycles) {
  asm volatile("" ::: "v109");  // force the hot kernel's 110-VGPR allocation
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin_cycles) __builtin_amdgcn_s_sleep(8);
  if ((threadIdx.x & 63) == 0) {
    const uint32_t w = blockIdx.x * 4 + threadIdx.x / 64;
    rec[2 * w] = hw;
    rec[2 * w + 1] = xcc;
  }
}

int main() {
  const int grid = 512, waves = grid * 4;
  uint32_t *d;
  CK(hipMalloc(&d, waves * 8));
  std::vector<uint32_t> h(waves * 2);
  for (size_t pad : {(size_t)0, (size_t)56 * 1024}) {
    CK(hipMemset(d, 0xff, waves * 8));
    hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), pad, 0, d, (uint64_t)2000000);  // 20 ms at the 100 MHz realtime clock
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, waves * 8, hipMemcpyDeviceToHost));
    std::map<uint32_t, int> wg_per_cu;  // key: xcc, se, sh, cu
    std::map<uint32_t, int> waves_per_simd;
    for (int w = 0; w < waves; ++w) {
      const uint32_t hw = h[2 * w], xcc = h[2 * w + 1] & 0xf;
      const uint32_t simd = (hw >> 4) & 3, cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const uint32_t key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
      if (w % 4 == 0) wg_per_cu[key]++;
      waves_per_simd[(key << 2) | simd]++;
    }
    std::map<int, int> hist, shist;
    for (auto &kv : wg_per_cu) hist[kv.second]++;
    for (auto &kv : waves_per_simd) shist[kv.second]++;
    printf("lds_pad %6zu B: %zu CUs used;", pad, wg_per_cu.size());
    for (auto &kv : hist) printf("  %d CUs with %d WG", kv.second, kv.first);
    printf("\n                 %zu SIMDs used;", waves_per_simd.size());
    for (auto &kv : shist) printf("  %d SIMDs with %d waves", kv.second, kv.first);
    printf("\n");
    fflush(stdout);
  }
  CK(hipFree(d));
  return 0;
}
