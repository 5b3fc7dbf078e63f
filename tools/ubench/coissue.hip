// coissue.hip -- does gfx950 co-issue VALU instructions of two waves sharing a
// SIMD (SQ_ACTIVE_INST_VALU2), and can the SHA-1 loop exploit it?
// Compute-only SHA-1 compression (production round code) with
//   mode 0: 256-thread workgroups, 2 workgroups/CU (today's hot-kernel shape)
//   mode 1: 512-thread workgroups (two waves of ONE workgroup per SIMD)
//   mode 2: mode 1 + s_barrier after every block (keeps the SIMD pair in lockstep)
//   mode 3: mode 2, odd waves of the pair delayed by half a block (stagger)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "sha1_device.h"

using namespace btsha1;

template <int MODE>
__global__ __launch_bounds__(512) void kern(uint32_t *out, int nblocks) {
  uint32_t h[5] = {kIV0, kIV1, kIV2, kIV3, kIV4};
  uint32_t m[16];
  for (int j = 0; j < 16; ++j) m[j] = (threadIdx.x + 1) * 2654435761u + j * 40503u + blockIdx.x;
  if constexpr (MODE == 3) {
    if ((threadIdx.x >> 6) >= 4) {  // waves 4-7: start half a block late
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = m[j];
      uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
      rounds_from<40>(w, a, b, c, d, e);
      h[0] ^= a;
    }
  }
  for (int blk = 0; blk < nblocks; ++blk) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(m[j] ^ blk);
    State st{h[0], h[1], h[2], h[3], h[4]};
    compress(st, w);
    h[0] = st.h0; h[1] = st.h1; h[2] = st.h2; h[3] = st.h3; h[4] = st.h4;
    if constexpr (MODE >= 2) __builtin_amdgcn_s_barrier();
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
}

template <int MODE>
void run(int waves_per_simd) {
  const int wg = MODE == 0 ? 256 : 512;
  const int threads = 256 * 4 * 64 * waves_per_simd;  // 256 CUs x 4 SIMDs x 64 lanes x waves
  const int blocks = threads / wg, nb = 3000;
  uint32_t *out;
  (void)hipMalloc(&out, (size_t)threads * 4);
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(wg), 0, 0, out, 50);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(wg), 0, 0, out, nb);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double gbs = (double)threads * nb * 64 / (best * 1e-3) / 1e9;
  printf("mode %d (wg %d) waves/SIMD=%d: %.3f ms, %.0f GB/s-equivalent\n", MODE, wg, waves_per_simd, best, gbs);
  (void)hipFree(out);
}

int main() {
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(2);
    run<1>(2);
    run<2>(2);
    run<3>(2);
  }
  run<0>(4);
  run<2>(4);
  return 0;
}
