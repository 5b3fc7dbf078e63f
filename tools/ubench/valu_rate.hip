// valu_rate.hip -- measures wave64 issue cost of the integer VALU ops the
// SHA-1 kernel is made of (gfx950), independent (8 chains) and dependent
// (1 chain), at 1..8 waves per SIMD, plus the in-kernel shader clock
// (s_memtime / s_memrealtime).  Informs the VALU roofline in DESIGN.md.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define OP_XOR "v_xor_b32 %0, %0, %1"
#define OP_ADD3 "v_add3_u32 %0, %0, %1, %0"
#define OP_ALIGN "v_alignbit_b32 %0, %0, %1, 7"
#define OP_BITOP3 "v_bitop3_b32 %0, %0, %1, %0 bitop3:0xca"
#define OP_PERM "v_perm_b32 %0, %0, %1, %2"
#define OP_FMA "v_fma_f32 %0, %0, %1, %0"
#define OP_PKFMA "v_pk_fma_f32 %0, %0, %1, %0"
#define OP_ADD "v_add_u32 %0, %0, %1"
#define OP_LSHR "v_lshrrev_b32 %0, 5, %0"
#define OP_LSHLOR "v_lshl_or_b32 %0, %0, 5, %1"
#define OP_LSHLADD "v_lshl_add_u32 %0, %0, 5, %1"
#define OP_OR3 "v_or3_b32 %0, %0, %1, %0"
#define OP_XAD "v_xad_u32 %0, %0, %1, %0"
#define OP_ANDOR "v_and_or_b32 %0, %0, %1, %0"
#define OP_BFI "v_bfi_b32 %0, %0, %1, %0"
#define OP_XOR64 "v_xor_b32 %0, %0, %1"

template <int KIND, int CHAINS>
__global__ __launch_bounds__(256) void kern(uint32_t *out, unsigned long long *clk, int iters) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i;
  uint32_t b = blockIdx.x | 1, sel = 0x00010203;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p[8];
  for (int i = 0; i < 8; ++i) p[i] = f2{(float)i, 1.0f};
  f2 pb = f2{1.0001f, 0.9999f};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int i = CHAINS == 1 ? 0 : c;
        if constexpr (KIND == 0) asm volatile(OP_XOR : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 1) asm volatile(OP_ADD3 : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 2) asm volatile(OP_ALIGN : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 3) asm volatile(OP_BITOP3 : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 4) asm volatile(OP_PERM : "+v"(a[i]) : "v"(b), "v"(sel));
        if constexpr (KIND == 5) asm volatile(OP_FMA : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 6) asm volatile(OP_PKFMA : "+v"(p[i]) : "v"(pb));
        if constexpr (KIND == 7) asm volatile(OP_ADD : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 8) asm volatile(OP_LSHR : "+v"(a[i]));
        if constexpr (KIND == 9) asm volatile(OP_LSHLOR : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 10) asm volatile(OP_LSHLADD : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 11) asm volatile(OP_OR3 : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 12) asm volatile(OP_XAD : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 13) asm volatile(OP_ANDOR : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 14) asm volatile(OP_BFI : "+v"(a[i]) : "v"(b));
        if constexpr (KIND == 15) {  // 50/50 mix: add3 + xor
          if (c & 1) asm volatile(OP_ADD3 : "+v"(a[i]) : "v"(b));
          else asm volatile(OP_XOR : "+v"(a[i]) : "v"(b));
        }
        if constexpr (KIND == 16) {  // 50/50 mix: alignbit + bitop3
          if (c & 1) asm volatile(OP_ALIGN : "+v"(a[i]) : "v"(b));
          else asm volatile(OP_BITOP3 : "+v"(a[i]) : "v"(b));
        }
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i] ^ __float_as_uint(p[i].x);
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int KIND, int CHAINS>
void run(const char *name, int waves_per_simd) {
  const int blocks = 256 * waves_per_simd;  // 256-thread blocks: 1 wave per SIMD each
  const int iters = 2000;
  uint32_t *out;
  unsigned long long *clk;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&clk, blocks * 16);
  hipLaunchKernelGGL((kern<KIND, CHAINS>), dim3(blocks), dim3(256), 0, 0, out, clk, 50);  // warm
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((kern<KIND, CHAINS>), dim3(blocks), dim3(256), 0, 0, out, clk, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(2 * blocks);
  hipMemcpy(h.data(), clk, blocks * 16, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < blocks; ++i) {
    cyc += h[2 * i];
    rt += h[2 * i + 1];
  }
  cyc /= blocks;
  rt /= blocks;
  const double ghz = cyc / (rt / 100e6) / 1e9;  // s_memrealtime ticks at 100 MHz
  const double instr_per_wave = (double)iters * 16 * 8;
  // per SIMD: waves_per_simd waves each issuing instr_per_wave
  const double cyc_per_instr_simd = cyc / (instr_per_wave * waves_per_simd);
  const double lane_ops = (double)blocks * 256 * instr_per_wave / (ms * 1e-3);
  printf("%-8s chains=%d waves/SIMD=%d: %.3f cyc/instr/SIMD (in-kernel clock %.2f GHz), %.1f T lane-ops/s, %.3f ms\n",
         name, CHAINS, waves_per_simd, cyc_per_instr_simd, ghz, lane_ops / 1e12, ms);
  hipFree(out);
  hipFree(clk);
}

int main() {
  for (int w : {2, 8}) {
    run<0, 8>("xor", w);
    run<7, 8>("add", w);
    run<8, 8>("lshrrev", w);
    run<9, 8>("lshl_or", w);
    run<10, 8>("lshl_add", w);
    run<11, 8>("or3", w);
    run<12, 8>("xad", w);
    run<13, 8>("and_or", w);
    run<14, 8>("bfi", w);
    run<1, 8>("add3", w);
    run<2, 8>("alignbit", w);
    run<3, 8>("bitop3", w);
    run<15, 8>("mix_add3_xor", w);
    run<16, 8>("mix_align_bitop3", w);
  }
  return 0;
}
