// sha1_order.hip -- does the ORDER of the 597 instructions of a block matter?
// pairing.hip shows the SIMD runs two waves fastest when both issue the same
// rate class together, and that full-rate ops grouped in runs (C8 C8 S8) beat
// the interleaved C C S pattern.  Here every instruction of the production
// block (shared-pair schedule, sha1_device.h) is an `asm volatile`, so the
// compiler keeps the written order, and the orders below are compared with the
// compiler's own schedule (variant 0) at 2 and 4 waves/SIMD, compute only.
//   1  natural: schedule word t, then round t
//   2  full-rate first: per round, f and the schedule's full-rate ops of word
//      t+LOOK together, then the round's and the word's rotates/adds
//   3  four-word groups: full-rate ops of 4 schedule words, their rotates,
//      then 4 rounds
// Prints GB/s-equivalent (64 B per block per lane) from wall time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "sha1_device.h"

using namespace btsha1;

__device__ __forceinline__ uint32_t X2(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int IMM>
__device__ __forceinline__ uint32_t B3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "i"(IMM));
  return r;
}
template <int N>  // rotate left by N
__device__ __forceinline__ uint32_t R(uint32_t a) {
  uint32_t r;
  asm volatile("v_alignbit_b32 %0, %1, %1, %2" : "=v"(r) : "v"(a), "i"(32 - N));
  return r;
}
__device__ __forceinline__ uint32_t A3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t A3s(uint32_t a, uint32_t b, uint32_t k) {
  uint32_t r;
  asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}
__device__ __forceinline__ uint32_t PERM(uint32_t a, uint32_t sel) {
  uint32_t r;
  asm volatile("v_perm_b32 %0, 0, %1, %2" : "=v"(r) : "v"(a), "s"(sel));
  return r;
}
__device__ __forceinline__ uint32_t ADD(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int T>
constexpr int fimm() { return T < 20 ? 0xCA : (T < 40 || T >= 60) ? 0x96 : 0xE8; }
template <int T>
constexpr uint32_t kconst() { return T < 20 ? 0x5a827999u : T < 40 ? 0x6ed9eba1u : T < 60 ? 0x8f1bbcdcu : 0xca62c1d6u; }

// Full schedule in W[80] (SSA values; the compiler keeps only what is live).
struct Blk {
  uint32_t W[80];
  uint32_t X[80];  // pre-rotation value of word t (t >= 16)
  uint32_t P[16];
  uint32_t a, b, c, d, e;
};

// full-rate part of schedule word t
template <int T>
__device__ __forceinline__ void sched_S(Blk &k) {
  if constexpr (T >= 16 && T < 32) {
    k.P[T - 16] = X2(k.W[T - 16], k.W[T - 8]);
    k.X[T] = B3<0x96>(k.P[T - 16], k.W[T - 3], k.W[T - 14]);
  } else if constexpr (T >= 32 && T < 64) {
    k.X[T] = X2(B3<0x96>(k.W[T - 3], k.W[T - 8], k.W[T - 14]), k.W[T - 16]);
  } else if constexpr (T >= 64 && T < 80) {
    k.X[T] = B3<0x96>(k.P[T - 64], k.W[T - 12], k.W[T - 32]);
  }
}
template <int T>
__device__ __forceinline__ void sched_C(Blk &k) {
  if constexpr (T >= 16 && T < 64) k.W[T] = R<1>(k.X[T]);
  else if constexpr (T >= 64 && T < 80) k.W[T] = R<4>(k.X[T]);
}
// round t split into its full-rate op (f) and the rest
template <int T>
__device__ __forceinline__ uint32_t round_S(Blk &k) { return B3<fimm<T>()>(k.b, k.c, k.d); }
template <int T>
__device__ __forceinline__ void round_C(Blk &k, uint32_t f) {
  const uint32_t r5 = R<5>(k.a);
  const uint32_t x = A3s(k.e, k.W[T], kconst<T>());
  const uint32_t t = A3(x, f, r5);
  k.e = k.d;
  k.d = k.c;
  k.c = R<30>(k.b);
  k.b = k.a;
  k.a = t;
}

template <int ORDER, int T>
__device__ __forceinline__ void step(Blk &k) {
  if constexpr (T < 80) {
    if constexpr (ORDER == 1) {
      sched_S<T>(k);
      sched_C<T>(k);
      const uint32_t f = round_S<T>(k);
      round_C<T>(k, f);
    } else if constexpr (ORDER == 2) {
      // word T+3 needs W[T] and older: computed at step T, used at round T+3
      const uint32_t f = round_S<T>(k);
      sched_S<T + 3>(k);
      round_C<T>(k, f);
      sched_C<T + 3>(k);
    } else if constexpr (ORDER == 3) {
      if constexpr (T % 4 == 0 && T >= 12) {
        // words T+4..T+7: full-rate parts of three, their rotates, then the fourth
        sched_S<T + 4>(k); sched_S<T + 5>(k); sched_S<T + 6>(k);
        sched_C<T + 4>(k); sched_C<T + 5>(k); sched_C<T + 6>(k);
        sched_S<T + 7>(k); sched_C<T + 7>(k);
      }
      const uint32_t f = round_S<T>(k);
      round_C<T>(k, f);
    }
    step<ORDER, T + 1>(k);
  }
}

template <int ORDER>
__device__ __forceinline__ void compress_ordered(uint32_t (&h)[5], const uint32_t (&m)[16], uint32_t sel) {
  Blk k;
#pragma unroll
  for (int j = 0; j < 16; ++j) k.W[j] = PERM(m[j], sel);
  k.a = h[0]; k.b = h[1]; k.c = h[2]; k.d = h[3]; k.e = h[4];
  step<ORDER, 0>(k);
  h[0] = ADD(h[0], k.a); h[1] = ADD(h[1], k.b); h[2] = ADD(h[2], k.c); h[3] = ADD(h[3], k.d); h[4] = ADD(h[4], k.e);
}

template <int V>
__global__ __launch_bounds__(256) void kern(uint32_t *out, int nblocks) {
  uint32_t h[5] = {kIV0, kIV1, kIV2, kIV3, kIV4};
  uint32_t m[16];
  for (int j = 0; j < 16; ++j) m[j] = (threadIdx.x + 1) * 2654435761u + j * 40503u + blockIdx.x;
  const uint32_t sel = __builtin_amdgcn_readfirstlane(0x00010203u + (uint32_t)(nblocks >> 30));
  for (int blk = 0; blk < nblocks; ++blk) {
    uint32_t mm[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) mm[j] = m[j] ^ (uint32_t)blk;
    if constexpr (V == 0) {
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = bswap(mm[j]);
      State st{h[0], h[1], h[2], h[3], h[4]};
      compress(st, w);
      h[0] = st.h0; h[1] = st.h1; h[2] = st.h2; h[3] = st.h3; h[4] = st.h4;
    } else {
      compress_ordered<V>(h, mm, sel);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
}

template <int V>
void run(int waves_per_simd, uint32_t *ref) {
  const int blocks = 256 * waves_per_simd, nb = 4000;
  uint32_t *out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, out, 100);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, out, nb);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  // same digests as variant 0?
  const size_t n = (size_t)blocks * 256;
  uint32_t *h = (uint32_t *)malloc(n * 4);
  (void)hipMemcpy(h, out, n * 4, hipMemcpyDeviceToHost);
  bool same = true;
  if (ref) for (size_t i = 0; i < n && same; ++i) same = h[i] == ref[i];
  if (!ref) same = true;
  printf("order %d waves/SIMD=%d: %.3f ms, %.0f GB/s-equivalent%s\n", V, waves_per_simd, best,
         (double)blocks * 256 * nb * 64 / (best * 1e-3) / 1e9, same ? "" : "  MISMATCH vs order 0");
  if (ref == nullptr && V == 0) {}
  free(h);
  (void)hipFree(out);
}

template <int V>
uint32_t *ref_of(int waves_per_simd) {
  const int blocks = 256 * waves_per_simd;
  uint32_t *out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, out, 4000);
  (void)hipDeviceSynchronize();
  uint32_t *h = (uint32_t *)malloc((size_t)blocks * 256 * 4);
  (void)hipMemcpy(h, out, (size_t)blocks * 256 * 4, hipMemcpyDeviceToHost);
  (void)hipFree(out);
  return h;
}

int main() {
  for (int w : {2, 4}) {
    uint32_t *ref = ref_of<0>(w);
    for (int rep = 0; rep < 2; ++rep) {
      run<0>(w, nullptr);
      run<1>(w, ref);
      run<2>(w, ref);
      run<3>(w, ref);
    }
    free(ref);
  }
  return 0;
}
