// sha1_alu.hip -- compute-only ceiling of the SHA-1 compression on gfx950:
// the production round code (csrc/sha1_device.h) run over register-resident
// message words, no memory traffic, at 1/2/4/8 waves per SIMD.  Compares with
// the hot kernel's measured rate to split "VALU issue" from "memory" costs.
// Variants: 0 = production compress; 1 = rotates as lshrrev + lshl_or;
// 2 = adds as VOP2 adds (no add3).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "sha1_device.h"

using namespace btsha1;

__device__ __forceinline__ uint32_t rot_lo(uint32_t x, int n) {
  uint32_t r;
  asm volatile("v_lshrrev_b32 %0, %1, %2\n\tv_lshl_or_b32 %0, %2, %3, %0" : "=&v"(r) : "i"(32 - n), "v"(x), "i"(n));
  return r;
}

template <int V, int T>
__device__ __forceinline__ void rnd(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e, uint32_t w) {
  if constexpr (V == 0) {
    sha1_round<T>(a, b, c, d, e, w);
  } else {
    uint32_t f, k;
    if constexpr (T < 20) { f = f_ch(b, c, d); k = 0x5a827999u; }
    else if constexpr (T < 40) { f = f_par(b, c, d); k = 0x6ed9eba1u; }
    else if constexpr (T < 60) { f = f_maj(b, c, d); k = 0x8f1bbcdcu; }
    else { f = f_par(b, c, d); k = 0xca62c1d6u; }
    uint32_t t;
    if constexpr (V == 1) t = rot_lo(a, 5) + f + (e + k + w);
    else {
      uint32_t s;
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(s) : "v"(e), "v"(w));
      asm volatile("v_add_u32 %0, %1, %0" : "+v"(s) : "s"(k));
      uint32_t r5 = rotl(a, 5);
      asm volatile("v_add_u32 %0, %1, %0" : "+v"(s) : "v"(f));
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(t) : "v"(r5), "v"(s));
    }
    e = d; d = c; c = (V == 1) ? rot_lo(b, 30) : rotl(b, 30); b = a; a = t;
  }
}

template <int V, int T>
__device__ __forceinline__ void rounds(uint32_t (&w)[16], uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e) {
  if constexpr (T < 80) {
    rnd<V, T>(a, b, c, d, e, sched<T>(w));
    rounds<V, T + 1>(w, a, b, c, d, e);
  }
}

// Variant 3: whole 80-word schedule first (S-op runs), then the 80 rounds.
template <int T>
__device__ __forceinline__ void sched_all(uint32_t (&w)[80]) {
  if constexpr (T < 80) {
    w[T] = rotl(__builtin_amdgcn_bitop3_b32(w[T - 3], w[T - 8], w[T - 14], 0x96) ^ w[T - 16], 1);
    sched_all<T + 1>(w);
  }
}
template <int T>
__device__ __forceinline__ void rounds_w80(const uint32_t (&w)[80], uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                           uint32_t &e) {
  if constexpr (T < 80) {
    sha1_round<T>(a, b, c, d, e, w[T]);
    rounds_w80<T + 1>(w, a, b, c, d, e);
  }
}

template <int V>
__global__ __launch_bounds__(256) void kern(uint32_t *out, unsigned long long *clk, int nblocks) {
  uint32_t h[5] = {kIV0, kIV1, kIV2, kIV3, kIV4};
  uint32_t m[16];
  for (int j = 0; j < 16; ++j) m[j] = (threadIdx.x + 1) * 2654435761u + j * 40503u + blockIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int blk = 0; blk < nblocks; ++blk) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(m[j] ^ blk);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    if constexpr (V == 3) {
      uint32_t w80[80];
#pragma unroll
      for (int j = 0; j < 16; ++j) w80[j] = w[j];
      sched_all<16>(w80);
      __builtin_amdgcn_sched_barrier(0);
      rounds_w80<0>(w80, a, b, c, d, e);
    } else {
      rounds<V, 0>(w, a, b, c, d, e);
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int V>
void run(int waves_per_simd, int ops_per_block) {
  const int blocks = 256 * waves_per_simd, nb = 4000;
  uint32_t *out; unsigned long long *clk;
  (void)hipMalloc(&out, blocks * 256 * 4);
  (void)hipMalloc(&clk, blocks * 16);
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, out, clk, 100);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, out, clk, nb);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> hc(2 * blocks);
  (void)hipMemcpy(hc.data(), clk, blocks * 16, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < blocks; ++i) { cyc += hc[2 * i]; rt += hc[2 * i + 1]; }
  cyc /= blocks; rt /= blocks;
  const double ghz = cyc / (rt / 100e6) / 1e9;
  const double gbs = (double)blocks * 256 * nb * 64 / (ms * 1e-3) / 1e9;
  printf("variant %d waves/SIMD=%d: %.2f cyc/block/wave, %.3f cyc/instr/SIMD (ops/block=%d), clock %.2f GHz, %.0f GB/s-equivalent\n",
         V, waves_per_simd, cyc / nb, cyc / nb / ops_per_block / waves_per_simd, ops_per_block, ghz, gbs);
  (void)hipFree(out); (void)hipFree(clk);
}

// `sha1_alu long N`: variant 0 at 2 waves/SIMD relaunched N times back to back
// (a sustained run for power/clock sampling); prints the mean GB/s-equivalent.
void run_long(int launches) {
  const int blocks = 512, nb = 4000;
  uint32_t *out; unsigned long long *clk;
  (void)hipMalloc(&out, blocks * 256 * 4);
  (void)hipMalloc(&clk, blocks * 16);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int i = 0; i < launches; ++i) hipLaunchKernelGGL(kern<0>, dim3(blocks), dim3(256), 0, 0, out, clk, nb);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  printf("long: %d launches, %.3f ms each, %.0f GB/s-equivalent\n", launches, ms / launches,
         (double)blocks * 256 * nb * 64 * launches / (ms * 1e-3) / 1e9);
  (void)hipFree(out); (void)hipFree(clk);
}

int main(int argc, char **argv) {
  if (argc > 2 && argv[1][0] == 'l') { run_long(atoi(argv[2])); return 0; }
  for (int rep = 0; rep < 2; ++rep)
    for (int w : {2, 4}) {
      run<0>(w, 613);
      run<3>(w, 613);
    }
  return 0;
}
