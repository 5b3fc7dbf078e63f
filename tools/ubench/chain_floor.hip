// chain_floor.hip -- where does the chain kernel's round wave (R of
// k_sha1_chain) spend its issue slots?  One wave per CU runs 8193 blocks of
// SHA-1 rounds (5 VALU per round, as in R) with the 80 W+K words per block
// taken from:
//   0  LDS, broadcast ds_read_b128, whole-block double buffering (production R)
//   1  SGPRs that never change (no loads at all: the VALU-only floor)
//   2  s_load_dwordx16 from global memory, one 16-word group ahead (offsets
//      in the instruction; one pointer add per block)
//   3  scalar loads per half block (16 + 16 + 8 words), one half ahead: each
//      lgkmcnt(0) wait comes 40 rounds after the loads it covers (SMEM
//      returns out of order, so only lgkmcnt(0) is a safe wait)
//   4  two ds_read_b128 per block (lanes 0..15 hold words 4L..4L+3, lanes
//      0..3 words 64..79) and a DPP row shift folded into one add per round
// Prints ms per chain and ns per block.  Compute only; the words are arbitrary.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "sha1_device.h"

using namespace btsha1;

constexpr int kBlocks = 8193;

template <int T>
__device__ __forceinline__ void rnd(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e, uint32_t wk) {
  uint32_t f;
  if constexpr (T < 20) f = f_ch(b, c, d);
  else if constexpr (T < 40) f = f_par(b, c, d);
  else if constexpr (T < 60) f = f_maj(b, c, d);
  else f = f_par(b, c, d);
  const uint32_t t = rotl(a, 5) + (f + e + wk);
  e = d;
  d = c;
  c = rotl(b, 30);
  b = a;
  a = t;
}

template <int T, int N>
__device__ __forceinline__ void rounds_v4(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                          const u32x4 (&q)[20]) {
  if constexpr (T < N) {
    const u32x4 v = q[T / 4];
    rnd<T>(a, b, c, d, e, v.x);
    rnd<T + 1>(a, b, c, d, e, v.y);
    rnd<T + 2>(a, b, c, d, e, v.z);
    rnd<T + 3>(a, b, c, d, e, v.w);
    rounds_v4<T + 4, N>(a, b, c, d, e, q);
  }
}

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

template <int T0, int J>
__device__ __forceinline__ void rounds_s16(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                           const u32x16 &g) {
  if constexpr (J < 16) {
    rnd<T0 + J>(a, b, c, d, e, g[J]);
    rounds_s16<T0, J + 1>(a, b, c, d, e, g);
  }
}

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

template <int T0, int J>
__device__ __forceinline__ void rounds_s8(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                          const u32x8 &g) {
  if constexpr (J < 8) {
    rnd<T0 + J>(a, b, c, d, e, g[J]);
    rounds_s8<T0, J + 1>(a, b, c, d, e, g);
  }
}

// 40 W+K words (half a block) in SGPRs: 16 + 16 + 8.
struct Half {
  u32x16 x, y;
  u32x8 z;
};

template <int OFF>
__device__ __forceinline__ u32x8 sload8(const uint32_t *p) {
  u32x8 v;
  asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(v) : "s"(p), "n"(OFF) : "memory");
  return v;
}

template <int OFF>  // byte offset, encoded in the instruction
__device__ __forceinline__ u32x16 sload16(const uint32_t *p) {
  u32x16 v;
  asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(v) : "s"(p), "n"(OFF) : "memory");
  return v;
}
__device__ __forceinline__ void swait(u32x16 &v) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(v)::"memory"); }
__device__ __forceinline__ void swait(Half &h) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(h.x), "+s"(h.y), "+s"(h.z)::"memory");
}
template <int OFF>
__device__ __forceinline__ Half sload_half(const uint32_t *p) {
  return Half{sload16<OFF>(p), sload16<OFF + 64>(p), sload8<OFF + 128>(p)};
}
template <int T0>
__device__ __forceinline__ void rounds_half(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                            const Half &h) {
  rounds_s16<T0, 0>(a, b, c, d, e, h.x);
  rounds_s16<T0 + 16, 0>(a, b, c, d, e, h.y);
  rounds_s8<T0 + 32, 0>(a, b, c, d, e, h.z);
}

// Mode 4: lane L (< 16) of the round wave holds W+K words 4L..4L+3 of the
// block (one ds_read_b128), lanes 0..3 words 64..79 (a second one); round t
// takes its word from lane t/4 through a DPP row shift folded into the add
// (v_add_u32_dpp ... row_shl:t/4), so lane 0 -- the lane whose digest is
// kept -- gets it with no extra instruction.  Other lanes compute garbage.
template <int T>
__device__ __forceinline__ uint32_t wk_dpp(const u32x4 &A, const u32x4 &B) {
  constexpr int g = T < 64 ? T / 4 : (T - 64) / 4;
  const uint32_t src = T < 64 ? A[T % 4] : B[T % 4];
  if constexpr (g == 0) return src;
  else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)src, 0x100 + g, 0xF, 0xF, false);
}

template <int T>
__device__ __forceinline__ void rnd_dpp(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                        const u32x4 &A, const u32x4 &B) {
  uint32_t f;
  if constexpr (T < 20) f = f_ch(b, c, d);
  else if constexpr (T < 40) f = f_par(b, c, d);
  else if constexpr (T < 60) f = f_maj(b, c, d);
  else f = f_par(b, c, d);
  const uint32_t t = rotl(a, 5) + f + (e + wk_dpp<T>(A, B));
  e = d;
  d = c;
  c = rotl(b, 30);
  b = a;
  a = t;
}

template <int T>
__device__ __forceinline__ void rounds_dpp(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                           const u32x4 &A, const u32x4 &B) {
  if constexpr (T < 80) {
    rnd_dpp<T>(a, b, c, d, e, A, B);
    rounds_dpp<T + 1>(a, b, c, d, e, A, B);
  }
}

template <int MODE>
__global__ __launch_bounds__(64) void kern(uint32_t *out, const uint32_t *wkmem) {
  __shared__ u32x4 lds[20 * 64];
  const uint32_t lane = threadIdx.x;
  uint32_t vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  for (int j = lane; j < 20 * 64; j += 64) lds[j] = u32x4{(uint32_t)j, (uint32_t)j * 3u, (uint32_t)j * 5u, (uint32_t)j * 7u};
  __syncthreads();
  uint32_t h0 = 0x67452301u + vzero, h1 = 0xefcdab89u + vzero, h2 = 0x98badcfeu + vzero, h3 = 0x10325476u + vzero,
           h4 = 0xc3d2e1f0u + vzero;
  if constexpr (MODE == 0) {
    const u32x4 *slot = lds + vzero;
    u32x4 wa[20], wb[20];
#pragma unroll
    for (int j = 0; j < 20; ++j) wa[j] = slot[j * 64];
    for (int k = 0; k < kBlocks; k += 2) {
#pragma unroll
      for (int j = 0; j < 20; ++j) wb[j] = slot[j * 64 + ((k + 1) & 63)];
      uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
      rounds_v4<0, 80>(a, b, c, d, e, wa);
      h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
#pragma unroll
      for (int j = 0; j < 20; ++j) wa[j] = slot[j * 64 + ((k + 2) & 63)];
      a = h0, b = h1, c = h2, d = h3, e = h4;
      rounds_v4<0, 80>(a, b, c, d, e, wb);
      h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
    }
  } else if constexpr (MODE == 1) {
    const uint32_t s = __builtin_amdgcn_readfirstlane(out[1]);  // opaque uniform word
    for (int k = 0; k < kBlocks; ++k) {
      uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
      u32x4 q[20];
#pragma unroll
      for (int j = 0; j < 20; ++j) q[j] = u32x4{s + j, s ^ j, s + 3 * j, s - j};
      rounds_v4<0, 80>(a, b, c, d, e, q);
      h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
    }
  } else if constexpr (MODE == 2) {
    // blocks of 80 words back to back; the pointer advances by one block per
    // iteration (one 64-bit SALU add)
    const uint32_t *p = wkmem;
    u32x16 g0 = sload16<0>(p);
    for (int k = 0; k < kBlocks; ++k) {
      uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
      swait(g0);
      u32x16 g1 = sload16<64>(p);
      rounds_s16<0, 0>(a, b, c, d, e, g0);
      swait(g1);
      u32x16 g2 = sload16<128>(p);
      rounds_s16<16, 0>(a, b, c, d, e, g1);
      swait(g2);
      u32x16 g3 = sload16<192>(p);
      rounds_s16<32, 0>(a, b, c, d, e, g2);
      swait(g3);
      u32x16 g4 = sload16<256>(p);
      rounds_s16<48, 0>(a, b, c, d, e, g3);
      swait(g4);
      g0 = sload16<320>(p);  // the next block's first group
      rounds_s16<64, 0>(a, b, c, d, e, g4);
      h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
      p += 80;
    }
    swait(g0);
  } else if constexpr (MODE == 4) {
    // block-major slot: block k's 80 words at lds[k*21 ..] (21 x 16 B stride)
    const uint32_t l16 = lane & 15u, l4 = lane & 3u;
    const u32x4 *blk = lds;
    u32x4 A = blk[l16], B = blk[16 + l4];
    for (int k = 0; k < kBlocks; ++k) {
      const u32x4 *nb = lds + ((k + 1) % 60) * 21;
      const u32x4 An = nb[l16], Bn = nb[16 + l4];
      uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
      rounds_dpp<0>(a, b, c, d, e, A, B);
      h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
      A = An;
      B = Bn;
    }
  } else if constexpr (MODE == 3) {
    // half-block segments: every wait is 40 rounds after the loads it covers
    const uint32_t *p = wkmem;
    Half lo = sload_half<0>(p);
    for (int k = 0; k < kBlocks; ++k) {
      uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
      swait(lo);
      Half hi = sload_half<160>(p);
      rounds_half<0>(a, b, c, d, e, lo);
      swait(hi);
      lo = sload_half<320>(p);  // next block's first half
      rounds_half<40>(a, b, c, d, e, hi);
      h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
      p += 80;
    }
    swait(lo);
  }
  if (lane == 0) out[blockIdx.x * 2] = h0 ^ h1 ^ h2 ^ h3 ^ h4;
}

template <int MODE>
void run(uint32_t *out, const uint32_t *wk, int wgs) {
  hipLaunchKernelGGL(kern<MODE>, dim3(wgs), dim3(64), 0, 0, out, wk);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern<MODE>, dim3(wgs), dim3(64), 0, 0, out, wk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const char *name[] = {"LDS broadcast ds_read_b128 (production R)", "SGPR constants (VALU-only floor)",
                        "s_load_dwordx16, one group ahead", "s_load, half-block segments",
                        "2 ds_read_b128 per block + DPP row shifts"};
  printf("mode %d %-44s workgroups=%d: %.3f ms per chain, %.1f ns per block\n", MODE, name[MODE], wgs, best,
         best * 1e6 / kBlocks);
}

int main() {
  uint32_t *out, *wk;
  (void)hipMalloc(&out, 4096 * 8);
  (void)hipMemset(out, 0, 4096 * 8);
  (void)hipMalloc(&wk, (kBlocks + 2) * 80 * 4);  // one 320-byte record per block, never reused
  (void)hipMemset(wk, 0x5a, (kBlocks + 2) * 80 * 4);
  for (int wgs : {1, 256}) {
    run<0>(out, wk, wgs);
    run<1>(out, wk, wgs);
    run<2>(out, wk, wgs);
    run<3>(out, wk, wgs);
    run<4>(out, wk, wgs);
  }
  return 0;
}
