// mixpattern.hip -- cost of mixing half-rate (C: v_add3/v_alignbit) and
// full-rate (S: v_xor/v_bitop3) VALU ops on gfx950, by ordering pattern.
// Each pattern string is issued over 8 independent register chains (no
// dependency stalls); we report wall cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define C1(r) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[r]) : "v"(b));
#define C2(r) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[r]) : "v"(b));
#define S1(r) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[r]) : "v"(b));
#define S3(r) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a[r]) : "v"(b));
#define S4(r) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[r]) : "v"(b));
#define S5(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[r]) : "v"(b));
#define S2(r) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0xca" : "+v"(a[r]) : "v"(b));

template <int P>
__global__ __launch_bounds__(256) void kern(uint32_t *out, int iters) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  uint32_t b = blockIdx.x | 1;
  for (int it = 0; it < iters; ++it) {
    // 24 instructions per pattern instance, chains rotate 0..7
    if constexpr (P == 0) { C1(0) C2(1) C1(2) C2(3) C1(4) C2(5) C1(6) C2(7) C1(0) C2(1) C1(2) C2(3) C1(4) C2(5) C1(6) C2(7) C1(0) C2(1) C1(2) C2(3) C1(4) C2(5) C1(6) C2(7) }
    if constexpr (P == 1) { S1(0) S2(1) S1(2) S2(3) S1(4) S2(5) S1(6) S2(7) S1(0) S2(1) S1(2) S2(3) S1(4) S2(5) S1(6) S2(7) S1(0) S2(1) S1(2) S2(3) S1(4) S2(5) S1(6) S2(7) }
    // 2:1 interleaved  C C S
    if constexpr (P == 2) { C1(0) C2(1) S1(2) C1(3) C2(4) S2(5) C1(6) C2(7) S1(0) C1(1) C2(2) S2(3) C1(4) C2(5) S1(6) C1(7) C2(0) S2(1) C1(2) C2(3) S1(4) C1(5) C2(6) S2(7) }
    // 2:1 grouped 16 C then 8 S
    if constexpr (P == 3) { C1(0) C2(1) C1(2) C2(3) C1(4) C2(5) C1(6) C2(7) C1(0) C2(1) C1(2) C2(3) C1(4) C2(5) C1(6) C2(7) S1(0) S2(1) S1(2) S2(3) S1(4) S2(5) S1(6) S2(7) }
    // 2:1 grouped by 4: CCCC CCCC SSSS
    if constexpr (P == 4) { C1(0) C2(1) C1(2) C2(3) C1(4) C2(5) C1(6) C2(7) S1(0) S2(1) S1(2) S2(3) C1(4) C2(5) C1(6) C2(7) C1(0) C2(1) C1(2) C2(3) S1(4) S2(5) S1(6) S2(7) }
    // 1:1 alternating
    if constexpr (P == 5) { C1(0) S1(1) C2(2) S2(3) C1(4) S1(5) C2(6) S2(7) C1(0) S1(1) C2(2) S2(3) C1(4) S1(5) C2(6) S2(7) C1(0) S1(1) C2(2) S2(3) C1(4) S1(5) C2(6) S2(7) }
    // 1:1 grouped 12 C then 12 S
    if constexpr (P == 6) { C1(0) C2(1) C1(2) C2(3) C1(4) C2(5) C1(6) C2(7) C1(0) C2(1) C1(2) C2(3) S1(4) S2(5) S1(6) S2(7) S1(0) S2(1) S1(2) S2(3) S1(4) S2(5) S1(6) S2(7) }
    // C S S (1:2)
    if constexpr (P == 7) { C1(0) S1(1) S2(2) C2(3) S1(4) S2(5) C1(6) S1(7) S2(0) C2(1) S1(2) S2(3) C1(4) S1(5) S2(6) C2(7) S1(0) S2(1) C1(2) S1(3) S2(4) C2(5) S1(6) S2(7) }
    if constexpr (P == 8) { S3(0) S3(1) S3(2) S3(3) S3(4) S3(5) S3(6) S3(7) S3(0) S3(1) S3(2) S3(3) S3(4) S3(5) S3(6) S3(7) S3(0) S3(1) S3(2) S3(3) S3(4) S3(5) S3(6) S3(7) }
    if constexpr (P == 9) { S1(0) S1(1) S1(2) S1(3) S1(4) S1(5) S1(6) S1(7) S1(0) S1(1) S1(2) S1(3) S1(4) S1(5) S1(6) S1(7) S1(0) S1(1) S1(2) S1(3) S1(4) S1(5) S1(6) S1(7) }
    if constexpr (P == 10) { S4(0) S4(1) S4(2) S4(3) S4(4) S4(5) S4(6) S4(7) S4(0) S4(1) S4(2) S4(3) S4(4) S4(5) S4(6) S4(7) S4(0) S4(1) S4(2) S4(3) S4(4) S4(5) S4(6) S4(7) }
    if constexpr (P == 11) { S5(0) S5(1) S5(2) S5(3) S5(4) S5(5) S5(6) S5(7) S5(0) S5(1) S5(2) S5(3) S5(4) S5(5) S5(6) S5(7) S5(0) S5(1) S5(2) S5(3) S5(4) S5(5) S5(6) S5(7) }
    if constexpr (P == 12) { S2(0) S2(1) S2(2) S2(3) S2(4) S2(5) S2(6) S2(7) S2(0) S2(1) S2(2) S2(3) S2(4) S2(5) S2(6) S2(7) S2(0) S2(1) S2(2) S2(3) S2(4) S2(5) S2(6) S2(7) }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int P>
void run(const char *name, int w) {
  const int blocks = 256 * w, iters = 20000;
  uint32_t *out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, out, 100);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern<P>, dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // instructions per SIMD = w waves * iters * 24; cycles at nominal 2.4 GHz (report ns too)
  const double ins = (double)w * iters * 24;
  printf("%-22s waves/SIMD=%d: %.3f ms, %.3f ns/instr/SIMD (= %.2f cyc @2.4GHz)\n", name, w, ms, ms * 1e6 / ins,
         ms * 1e6 / ins * 2.4);
  (void)hipFree(out);
}

int main() {
  for (int w : {1, 2, 4, 8}) {
    run<9>("xor e32 (4B)", w);
    run<8>("xor e64 (8B)", w);
    run<11>("add e32 (4B)", w);
    run<10>("add e64 (8B)", w);
    run<12>("bitop3 (8B)", w);
    run<0>("allC", w);
  }
  return 0;
}
