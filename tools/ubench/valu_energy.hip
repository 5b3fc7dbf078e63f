// valu_energy.hip -- board power per VALU instruction class on gfx950.
// The hot kernel is capped by board power, so what an
// instruction COSTS in energy matters as much as its issue slots.  Each mode
// runs one instruction class in 8 independent dependency chains per lane, on
// 8 waves per SIMD, with SHA-like random operands, for ~4 s; board power is
// sampled beside it (tools/gpu_session.sh power_valu).  Prints the per-mode
// wave-instruction rate and the wall-clock window.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <ctime>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int M>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  if constexpr (M == 0) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  else if constexpr (M == 1) asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  else if constexpr (M == 2) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  else if constexpr (M == 3) asm volatile("v_alignbit_b32 %0, %1, %1, 27" : "=v"(r) : "v"(a));
  else if constexpr (M == 4) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  else if constexpr (M == 5) asm volatile("v_perm_b32 %0, 0, %1, %2" : "=v"(r) : "v"(a), "s"(0x00010203u));
  else if constexpr (M == 6) asm volatile("v_lshl_or_b32 %0, %1, 5, %2" : "=v"(r) : "v"(a), "v"(b));
  else asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

template <int M>
__global__ __launch_bounds__(256) void kern(uint32_t *out, int iters) {
  uint32_t x[8], y = threadIdx.x * 0x9E3779B9u + blockIdx.x, z = y * 0x85EBCA6Bu;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (y + j) * 0xC2B2AE35u ^ z;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = op<M>(x[j], x[(j + 1) & 7], x[(j + 3) & 7]);
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= x[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int M>
void run(const char *name, uint32_t *out, double seconds) {
  const int blocks = 256 * 8;  // 8 waves per SIMD
  // calibrate on a short launch
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int cal = 200;
  hipLaunchKernelGGL(kern<M>, dim3(blocks), dim3(256), 0, 0, out, cal);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern<M>, dim3(blocks), dim3(256), 0, 0, out, cal);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const int iters = (int)(cal * 100.0 / ms);  // ~100 ms launches
  const int launches = (int)(seconds * 10);
  const time_t t0 = time(nullptr);
  CK(hipEventRecord(e0));
  for (int l = 0; l < launches; ++l) hipLaunchKernelGGL(kern<M>, dim3(blocks), dim3(256), 0, 0, out, iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const time_t t1 = time(nullptr);
  const double winst = (double)blocks * 4 * iters * 16 * 8 * launches;  // wave-instructions
  char ts[2][16];
  strftime(ts[0], sizeof ts[0], "%H:%M:%S", localtime(&t0));
  strftime(ts[1], sizeof ts[1], "%H:%M:%S", localtime(&t1));
  printf("%-10s %8.3f G wave-instr/s  (%.3f ns per instr per SIMD)  [%s - %s]\n", name, winst / (ms * 1e-3) / 1e9,
         ms * 1e-3 / (winst / 1024) * 1e9, ts[0], ts[1]);
  fflush(stdout);
}

int main(int argc, char **argv) {
  const double sec = argc > 1 ? atof(argv[1]) : 4.0;
  uint32_t *out;
  CK(hipMalloc(&out, 256 * 8 * 256 * 4));
  run<0>("xor", out, sec);
  run<1>("add", out, sec);
  run<2>("add3", out, sec);
  run<3>("alignbit", out, sec);
  run<4>("bitop3", out, sec);
  run<5>("perm", out, sec);
  run<6>("lshl_or", out, sec);
  run<7>("mov", out, sec);
  CK(hipFree(out));
  return 0;
}
