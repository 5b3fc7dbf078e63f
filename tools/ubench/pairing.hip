// pairing.hip -- which VALU instructions of two waves sharing a SIMD issue in
// the same slot on gfx950?  512-thread workgroups (8 waves, two per SIMD), one
// workgroup per CU.  Each wave runs 8 independent chains of one of:
//   S = v_xor_b32 (full-rate class), C = v_add3_u32 (half-rate class).
// Modes: 0 all S | 1 all C | 2 waves 0-3 S, 4-7 C | 3 even waves S, odd C |
//        4 every wave alternates C,S | 5 all v_bitop3 | 6 waves 0-3 bitop3, 4-7 add3
// Run under rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 to see co-issue.
#include <hip/hip_runtime.h>
#include <cstdio>

#define S(r) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[r]) : "v"(b));
#define B(r) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a[r]) : "v"(b));
#define C(r) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[r]) : "v"(b));
#define S8 S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)
#define B8 B(0) B(1) B(2) B(3) B(4) B(5) B(6) B(7)
#define C8 C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7)
#define CS8 C(0) S(1) C(2) S(3) C(4) S(5) C(6) S(7)

#define CSS8 C(0) S(1) S(2) C(3) S(4) S(5) C(6) S(7)
#define CCSS8 C(0) C(1) S(2) S(3) C(4) C(5) S(6) S(7)
#define CCS8 C(0) C(1) S(2) C(3) C(4) S(5) C(6) C(7)
#define S1CH S(0) S(0) S(0) S(0) S(0) S(0) S(0) S(0)
#define S2CH S(0) S(1) S(0) S(1) S(0) S(1) S(0) S(1)
#define CB8 C(0) B(1) C(2) B(3) C(4) B(5) C(6) B(7)
#define CCB8 C(0) C(1) B(2) C(3) C(4) B(5) C(6) C(7)
#define CCCCB C(0) C(1) C(2) C(3) B(4)

template <int M>
__global__ __launch_bounds__(512) void kern(uint32_t *out, int iters) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  uint32_t b = blockIdx.x | 1;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  bool s_wave;
  if constexpr (M == 0 || M == 5) s_wave = true;
  else if constexpr (M == 13 || M == 15 || M == 16) s_wave = w < 4;
  else if constexpr (M == 1) s_wave = false;
  else if constexpr (M == 2 || M == 6) s_wave = w < 4;
  else s_wave = (w & 1) == 0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (M == 4) {
      CS8 CS8 CS8
    } else if constexpr (M == 7) {
      CSS8 CSS8 CSS8
    } else if constexpr (M == 8) {
      CCSS8 CCSS8 CCSS8
    } else if constexpr (M == 9) {
      CCS8 CCS8 CCS8
    } else if constexpr (M == 10) {
      S1CH S1CH S1CH
    } else if constexpr (M == 11) {
      S2CH S2CH S2CH
    } else if constexpr (M == 12) {
      CB8 CB8 CB8
    } else if constexpr (M == 13) {
      if (s_wave) { CS8 CS8 CS8 } else { S(0) CS8 CS8 CS8 }  // SIMD partner offset by one
    } else if constexpr (M == 14) {
      C8 C8 S8                                               // 2:1, grouped runs
    } else if constexpr (M == 15) {
      if (s_wave) { CCS8 CCS8 CCS8 } else { C(7) CCS8 CCS8 C(0) C(1) S(2) C(3) C(4) S(5) C(6) }  // partner shifted by one
    } else if constexpr (M == 16) {
      if (s_wave) { C8 C8 S8 } else { S8 C8 C8 }             // grouped, partner in the other phase
    } else if constexpr (M == 17) {
      CCB8 CCB8 CCB8                                         // 2:1 with bitop3 as the full-rate op
    } else if constexpr (M == 18) {
      CCCCB CCCCB CCCCB CCCCB C(0) C(1) C(2) C(3)            // the round's 4:1 (24 instr)
    } else if constexpr (M == 5) {
      B8 B8 B8
    } else if constexpr (M == 6) {
      if (s_wave) { B8 B8 B8 } else { C8 C8 C8 }
    } else {
      if (s_wave) { S8 S8 S8 } else { C8 C8 C8 }
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int M>
void run(const char *name) {
  const int blocks = 256, iters = 40000;
  uint32_t *out;
  (void)hipMalloc(&out, blocks * 512 * 4);
  hipLaunchKernelGGL(kern<M>, dim3(blocks), dim3(512), 0, 0, out, 100);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern<M>, dim3(blocks), dim3(512), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double ins = 2.0 * iters * 24;  // per SIMD: 2 waves
  printf("mode %d %-28s %.3f ms  %.3f ns/instr/SIMD\n", M, name, ms, ms * 1e6 / ins);
  (void)hipFree(out);
}

int main() {
  run<0>("all xor");
  run<1>("all add3");
  run<2>("waves0-3 xor, 4-7 add3");
  run<3>("even xor, odd add3");
  run<4>("all alternate add3,xor");
  run<5>("all bitop3");
  run<6>("waves0-3 bitop3, 4-7 add3");
  run<7>("all C S S");
  run<8>("all C C S S");
  run<9>("all C C S (SHA-1 ratio)");
  run<10>("all xor, 1 dependent chain");
  run<11>("all xor, 2 chains");
  run<12>("all alternate add3,bitop3");
  run<13>("C,S alt; waves4-7 offset 1");
  run<14>("C8 C8 S8 grouped (2:1)");
  run<15>("C C S, partner offset 1");
  run<16>("C8C8S8 vs S8C8C8 partner");
  run<17>("C C bitop3 (2:1)");
  run<18>("(C C C C bitop3) rounds 4:1");
  return 0;
}
