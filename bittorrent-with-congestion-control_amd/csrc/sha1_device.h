// sha1_device.h -- SHA-1 compression for CDNA4 (gfx950), one message per lane.
//
// Device restatement of the reference's SHA1Guts (sha.c:176-451).  Arithmetic
// is identical (FIPS 180-1); the structure is not:
//   * the 80-word schedule buf[80] (sha.c:179,191-200) becomes a 16-word
//     rolling window held in VGPRs, expanded just in time inside the rounds;
//   * the round functions F_0_19 / F_20_39 / F_40_59 / F_60_79 (sha.c:52-55)
//     are each ONE v_bitop3_b32 (gfx950 three-input truth-table op):
//     Ch = 0xCA, Parity = 0x96, Maj = 0xE8 over (b, c, d);
//   * ROTL (sha.c:49) is v_alignbit_b32, BYTESWAP (sha.c:80-81) is v_perm_b32,
//     and the five-term sum of DO_ROUND (sha.c:57-64) is two v_add3_u32.
//   * the schedule shares 16 XOR pairs between words 16..31 and 64..79 via the
//     recurrence squared twice (sched_pair below).
// Per 64-byte block: 80 x 5 round ops + 176 schedule ops (48 x 3 + 16 x 2) +
// 16 byte swaps + 5 state adds = 597 VALU instructions (613 with the plain
// recurrence); no memory traffic besides the block.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace btsha1 {

constexpr uint32_t kIV0 = 0x67452301u, kIV1 = 0xefcdab89u, kIV2 = 0x98badcfeu,
                   kIV3 = 0x10325476u, kIV4 = 0xc3d2e1f0u;  // sha.c:155-159

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_rotateleft32(x, n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// bitop3 truth-table index = (S0 << 2) | (S1 << 1) | S2.
__device__ __forceinline__ uint32_t f_ch(uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);  // d ^ (b & (c ^ d))   sha.c:52
}
__device__ __forceinline__ uint32_t f_par(uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);  // b ^ c ^ d          sha.c:53,55
}
__device__ __forceinline__ uint32_t f_maj(uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);  // (b&(c|d)) | (c&d)  sha.c:54
}

struct State {
  uint32_t h0, h1, h2, h3, h4;
  __device__ __forceinline__ void init() {
    h0 = kIV0; h1 = kIV1; h2 = kIV2; h3 = kIV3; h4 = kIV4;
  }
};

template <int T>
__device__ __forceinline__ void sha1_round(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                           uint32_t &e, uint32_t w) {
  uint32_t f, k;
  if constexpr (T < 20) {
    f = f_ch(b, c, d);
    k = 0x5a827999u;  // sha.c:66
  } else if constexpr (T < 40) {
    f = f_par(b, c, d);
    k = 0x6ed9eba1u;  // sha.c:67
  } else if constexpr (T < 60) {
    f = f_maj(b, c, d);
    k = 0x8f1bbcdcu;  // sha.c:68
  } else {
    f = f_par(b, c, d);
    k = 0xca62c1d6u;  // sha.c:69
  }
  const uint32_t t = rotl(a, 5) + f + (e + k + w);
  e = d;
  d = c;
  c = rotl(b, 30);
  b = a;
  a = t;
}

// Schedule word t >= 16 in the rolling window (sha.c:196-200):
// W[t] = ROTL1(W[t-3] ^ W[t-8] ^ W[t-14] ^ W[t-16]); W[t-16] lives in slot t&15.
template <int T>
__device__ __forceinline__ uint32_t sched(uint32_t (&w)[16]) {
  if constexpr (T >= 16) {
    w[T & 15] = rotl(__builtin_amdgcn_bitop3_b32(w[(T - 3) & 15], w[(T - 8) & 15], w[(T - 14) & 15], 0x96) ^
                         w[T & 15],
                     1);
  }
  return w[T & 15];
}

template <int T>
__device__ __forceinline__ void rounds_from(uint32_t (&w)[16], uint32_t &a, uint32_t &b, uint32_t &c,
                                            uint32_t &d, uint32_t &e) {
  if constexpr (T < 80) {
    sha1_round<T>(a, b, c, d, e, sched<T>(w));
    rounds_from<T + 1>(w, a, b, c, d, e);
  }
}

// Schedule with shared pairs (597 instead of 613 VALU per block; measured
// +1.4 % on the power-capped hot kernel, profiles/r01/experiments.md).  The
// recurrence squared twice over GF(2) gives, for t >= 64,
//   W[t] = ROTL4(W[t-12] ^ W[t-32] ^ W[t-56] ^ W[t-64]),
// and its pair W[t-64] ^ W[t-56] = W[i] ^ W[i+8] (i = t-64) is exactly the
// pair W[t'-16] ^ W[t'-8] that word t' = i+16 needs.  So words 16..31 keep
// their pair P[i] and words 64..79 cost bitop3 + rotate instead of
// xor + bitop3 + rotate.  Q[i] = W[32+i] stays live for those words too
// (~32 VGPRs more; occupancy is set by the chunk count, not registers).
template <int T>
__device__ __forceinline__ uint32_t sched_pair(uint32_t (&w)[16], uint32_t (&p)[16], uint32_t (&q)[16]) {
  if constexpr (T >= 16 && T < 32) {
    p[T - 16] = w[T & 15] ^ w[(T - 8) & 15];
    w[T & 15] = rotl(__builtin_amdgcn_bitop3_b32(p[T - 16], w[(T - 3) & 15], w[(T - 14) & 15], 0x96), 1);
  } else if constexpr (T >= 32 && T < 64) {
    sched<T>(w);
    if constexpr (T < 48) q[T - 32] = w[T & 15];
  } else if constexpr (T >= 64) {
    w[T & 15] = rotl(__builtin_amdgcn_bitop3_b32(p[T - 64], w[(T - 12) & 15], q[T - 64], 0x96), 4);
  }
  return w[T & 15];
}

template <int T>
__device__ __forceinline__ void rounds_pair_from(uint32_t (&w)[16], uint32_t (&p)[16], uint32_t (&q)[16],
                                                 uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e) {
  if constexpr (T < 80) {
    sha1_round<T>(a, b, c, d, e, sched_pair<T>(w, p, q));
    rounds_pair_from<T + 1>(w, p, q, a, b, c, d, e);
  }
}

// One compression of the 16 big-endian message words w (clobbered).
__device__ __forceinline__ void compress(State &s, uint32_t (&w)[16]) {
  uint32_t a = s.h0, b = s.h1, c = s.h2, d = s.h3, e = s.h4;
  uint32_t p[16], q[16];
  rounds_pair_from<0>(w, p, q, a, b, c, d, e);
  s.h0 += a;  // sha.c:446-450
  s.h1 += b;
  s.h2 += c;
  s.h3 += d;
  s.h4 += e;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Four little-endian 16-byte loads -> 16 big-endian words (sha.c:186-189).
__device__ __forceinline__ void block_from_le(uint32_t (&w)[16], const u32x4 &q0, const u32x4 &q1,
                                              const u32x4 &q2, const u32x4 &q3) {
  w[0] = bswap(q0.x); w[1] = bswap(q0.y); w[2] = bswap(q0.z); w[3] = bswap(q0.w);
  w[4] = bswap(q1.x); w[5] = bswap(q1.y); w[6] = bswap(q1.z); w[7] = bswap(q1.w);
  w[8] = bswap(q2.x); w[9] = bswap(q2.y); w[10] = bswap(q2.z); w[11] = bswap(q2.w);
  w[12] = bswap(q3.x); w[13] = bswap(q3.y); w[14] = bswap(q3.z); w[15] = bswap(q3.w);
}

// Final block(s) of a message (sha.c:529-543): `tail` holds the r = len % 64
// trailing message bytes as big-endian words (bytes past r already zero).
// Appends 0x80, zero fill and the 64-bit big-endian bit count, compressing one
// block when r <= 55 and two otherwise.
__device__ __forceinline__ void finish(State &s, uint32_t (&tail)[16], uint32_t r, uint64_t len_bytes) {
  const uint32_t wi = r >> 2;
  const uint32_t mark = 0x80000000u >> ((r & 3) * 8);
#pragma unroll
  for (int j = 0; j < 16; ++j) tail[j] |= (j == (int)wi) ? mark : 0u;
  const uint64_t bits = len_bytes * 8ull;
  if (r >= 56) {
    compress(s, tail);
#pragma unroll
    for (int j = 0; j < 16; ++j) tail[j] = 0u;
  }
  tail[14] = (uint32_t)(bits >> 32);
  tail[15] = (uint32_t)bits;
  compress(s, tail);
}

// Keep the first `nbytes` (0..4) bytes of a big-endian word.
__device__ __forceinline__ uint32_t keep_be_bytes(uint32_t v, uint32_t nbytes) {
  return nbytes >= 4 ? v : (nbytes == 0 ? 0u : (v & (0xFFFFFFFFu << (32 - 8 * nbytes))));
}

}  // namespace btsha1
