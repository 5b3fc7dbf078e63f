// sha1_kernels.hip -- gfx950 kernels of the SHA-1 chunk path + their launchers.
//
// SHA-1 is a serial Merkle-Damgard chain (SURVEY.md §7 "Serial chain"), so
// parallelism is across messages only.  The throughput kernels give each lane
// one message; the latency kernels split one chain's work between a loader /
// schedule wave S and a round wave R that meet in LDS.  Which kernel a batch
// runs follows from its size and the device's CU count.
//   k_sha1_fixed    the hot path: n equal-length chunks at a fixed pitch in HBM
//                   (make_chunks' 512 KiB chunks, chunk.c:20-21; received-chunk
//                   verify, util.c:311-313, when VERIFY).  Each lane streams its
//                   own chunk through a register ring of NBUF 128-byte lines,
//                   issuing line i+NBUF-1 while compressing line i, so HBM
//                   latency hides inside one wave (only 2 waves/SIMD exist at
//                   131072 chunks).  Loads are raw buffer loads off a per-wave
//                   descriptor: per-lane 32-bit voffset = lane * pitch, the
//                   line offset rides in the scalar soffset -> zero VALU
//                   address arithmetic in the loop.
//   k_sha1_lds      the hot path with coalesced LDS-DMA staging (a rejected
//                   variant: built only into the experiments library).
//   k_sha1_lat      small fixed-layout batches (<= 128 chunks per CU, 32768 on
//                   MI355X: small verify batches): a loader/schedule wave and a round
//                   wave per 64 chunks meet in LDS, cutting a lone chain's
//                   instruction count from 597 to ~426 per block.
//   k_sha1_chain    ONE message per two-wave workgroup (<= 2 chunks per CU;
//                   shahash, SHA1Update/SHA1Final midstates): S prepares 64 of
//                   the message's blocks at a time, R runs them back to back.
//   k_sha1_lat_ragged  k_sha1_lat's split for 64 messages of any lengths and
//                   alignment (ragged batches of 2 .. 128 per CU).
//   k_sha1_ragged   arbitrary (offset, length) messages and layouts the
//                   fixed kernels do not take (pitch not a 16-byte multiple,
//                   offsets past 4 GiB per wave), one message per lane.
//   k_fill_synthetic  frozen counter-based generator (bench/test data in HBM).
//   k_lookup_build / k_lookup_query  digest -> first index table in HBM
//                   (get_chunk_id / find_chunk, util.c:3-39).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha1_device.h"
#include "sha1_launch.h"

namespace btsha1 {

constexpr int kBlock = 256;  // 4 waves; 2 blocks per CU at 131072 chunks

// ---------------------------------------------------------------------------
// Hot path.
// ---------------------------------------------------------------------------
// One ring slot = L consecutive 128-byte lines of the lane's own chunk
// (2L SHA-1 blocks), fetched as 8L back-to-back 16-byte buffer loads so the
// DRAM sees one L*128-byte burst per chunk per slot.
template <int L, int AUX>
__device__ __forceinline__ void load_slot(u32x4 (&q)[8 * L], __amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                          uint32_t soff) {
#pragma unroll
  for (int j = 0; j < 8 * L; ++j) q[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff + 16 * j, AUX);
}

template <int L>
__device__ __forceinline__ void compress_slot(State &st, const u32x4 (&q)[8 * L]) {
#pragma unroll
  for (int b = 0; b < 2 * L; ++b) {
    uint32_t w[16];
    block_from_le(w, q[4 * b], q[4 * b + 1], q[4 * b + 2], q[4 * b + 3]);
    compress(st, w);
  }
}

// The r = len % 64 trailing bytes of the lane's chunk as big-endian words,
// bytes past r zero (4-byte buffer loads, range-checked).
__device__ __forceinline__ void load_tail(uint32_t (&tail)[16], __amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                          uint32_t nblocks, uint32_t r) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t have = r > 4u * j ? r - 4u * j : 0u;
    uint32_t v = 0;
    if (have) v = keep_be_bytes(bswap(__builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, nblocks * 64u + 4u * j, 0)), have);
    tail[j] = v;
  }
}

// Digest store (sha.c:550-553 big-endian bytes) and the optional fused
// compare of util.c:311-313, for the lanes that own a chunk.
template <bool VERIFY>
__device__ __forceinline__ void store_digest(const State &st, uint32_t lane, uint32_t nvalid, uint64_t chunk0,
                                             uint8_t *__restrict__ digests, const uint8_t *__restrict__ expected,
                                             uint8_t *__restrict__ ok) {
  if (lane < nvalid) {
    const uint64_t idx = chunk0 + lane;
    const uint32_t d0 = bswap(st.h0), d1 = bswap(st.h1), d2 = bswap(st.h2), d3 = bswap(st.h3), d4 = bswap(st.h4);
    if (digests) {
      uint32_t *o = (uint32_t *)(digests + idx * 20u);
      o[0] = d0; o[1] = d1; o[2] = d2; o[3] = d3; o[4] = d4;
    }
    if constexpr (VERIFY) {  // memcmp(hash, chunk->hash, 20) == 0
      const uint8_t *x = expected + idx * 20u;
      uint32_t e[5];
#pragma unroll
      for (int k = 0; k < 5; ++k)
        e[k] = (uint32_t)x[4 * k] | ((uint32_t)x[4 * k + 1] << 8) | ((uint32_t)x[4 * k + 2] << 16) |
               ((uint32_t)x[4 * k + 3] << 24);
      ok[idx] = (uint8_t)((e[0] == d0) & (e[1] == d1) & (e[2] == d2) & (e[3] == d3) & (e[4] == d4));
    }
  }
}

// Shared tail of the fixed-layout kernels: whole blocks from `done` on (fewer
// than one ring turn), the tail bytes + MD padding, the digest store and the
// optional fused compare.
template <bool VERIFY>
__device__ __forceinline__ void epilogue(State &st, __amdgpu_buffer_rsrc_t rsrc, uint32_t voff, uint32_t done,
                                         uint32_t len, uint32_t lane, uint32_t nvalid, uint64_t chunk0,
                                         uint8_t *__restrict__ digests, const uint8_t *__restrict__ expected,
                                         uint8_t *__restrict__ ok) {
  const uint32_t nblocks = len >> 6;
  for (uint32_t b = done; b < nblocks; ++b) {
    uint32_t w[16];
    const uint32_t o = b * 64u;
    block_from_le(w, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, o, 0),
                  __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, o + 16, 0),
                  __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, o + 32, 0),
                  __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, o + 48, 0));
    compress(st, w);
  }
  // Tail bytes + MD padding (sha.c:536-543); r is uniform across the batch.
  const uint32_t r = len & 63u;
  uint32_t tail[16];
  load_tail(tail, rsrc, voff, nblocks, r);
  finish(st, tail, r, len);
  store_digest<VERIFY>(st, lane, nvalid, chunk0, digests, expected, ok);
}

// NBUF ring slots of L lines; AUX = buffer-load cache policy (0 default, 2 nt).
// tail_len != 0: one more, shorter chunk follows the n_chunks full ones (the
// last fread of make_chunks, chunk.c:20); the first wave past the full ones
// (chunk0 = n_chunks rounded up to 64) hashes it alone, inside the same launch,
// so its chain runs beside the full chunks' instead of after them.
// In-kernel clock stamp (MI355X_MICROARCH.md "DVFS give-back" item 6): the
// shader-clock counter and the constant-rate real-time counter, each read with
// its lgkmcnt wait inside one asm statement, fenced against code motion.
struct Stamp {
  uint64_t mem, real;
};
__device__ __forceinline__ Stamp take_stamp() {
  Stamp t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t.mem), "=s"(t.real)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// STAMP (diagnostic build only, btsha1_launch_fixed_stamped): lane 0 of each
// wave stores {memtime, realtime} before and after the main loop to
// stamps[4*wave ..] through ordinary vector stores.  The production kernel is
// the STAMP = false instantiation, in which no stamp executes.
template <int NBUF, int L, int AUX, bool VERIFY, bool STAMP = false>
__global__ __launch_bounds__(kBlock, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_sha1_fixed(
    const uint8_t *__restrict__ base, uint64_t n_chunks, uint32_t pitch, uint32_t len, uint8_t *__restrict__ digests,
    const uint8_t *__restrict__ expected, uint8_t *__restrict__ ok, uint32_t tail_len, uint64_t *__restrict__ stamps) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint64_t chunk0 = (uint64_t)blockIdx.x * blockDim.x + (uint64_t)wave * 64u;  // wave-uniform
  uint32_t nvalid;
  if (chunk0 < n_chunks) {
    const uint64_t left = n_chunks - chunk0;
    nvalid = left < 64 ? (uint32_t)left : 64u;
  } else {
    if (tail_len == 0 || chunk0 != ((n_chunks + 63u) & ~(uint64_t)63u)) return;
    chunk0 = n_chunks;  // the tail chunk: digest index n_chunks, bytes at n_chunks * pitch
    nvalid = 1;
    len = tail_len;
  }
  // Lanes past the end re-hash the wave's last chunk (no divergence, no store).
  const uint32_t mine = lane < nvalid ? lane : nvalid - 1u;
  const uint32_t voff = mine * pitch;
  // Bytes this wave may read; the host guarantees 64*pitch + 4096 <= 2^32.
  const uint32_t nrec = (nvalid - 1u) * pitch + ((len + 3u) & ~3u);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void *)(base + chunk0 * (uint64_t)pitch), (short)0, (int)nrec, 0x00020000);

  State st;
  st.init();
  constexpr uint32_t kSlot = 128u * L;
  const uint32_t nblocks = len >> 6;
  const uint32_t nslots = nblocks / (2u * L);
  const uint32_t nmain = (nslots / NBUF) * NBUF;  // slots covered by the pipelined loop

  Stamp t0{};
  if constexpr (STAMP) t0 = take_stamp();
  if (nmain) {
    u32x4 ring[NBUF][8 * L];
#pragma unroll
    for (int i = 0; i < NBUF - 1; ++i) load_slot<L, AUX>(ring[i], rsrc, voff, (uint32_t)i * kSlot);
    for (uint32_t slot = 0; slot < nmain; slot += NBUF) {
#pragma unroll
      for (int s = 0; s < NBUF; ++s) {
        // Prefetch may run NBUF-1 slots past the chunk: it reads the next
        // chunk's bytes or, past nrec, range-checked zeros; never used.
        load_slot<L, AUX>(ring[(s + NBUF - 1) % NBUF], rsrc, voff, (slot + s + NBUF - 1) * kSlot);
        // Pin the prefetch here: left alone, the scheduler sinks it to the
        // loop end to cut register pressure and the ring degenerates into a
        // vmcnt(0) at the loop head.
        __builtin_amdgcn_sched_barrier(0);
        compress_slot<L>(st, ring[s]);
      }
    }
  }
  if constexpr (STAMP) {
    const Stamp t1 = take_stamp();
    if (lane == 0) {
      uint64_t *o = stamps + 4 * (chunk0 >> 6);
      o[0] = t0.mem;
      o[1] = t0.real;
      o[2] = t1.mem;
      o[3] = t1.real;
    }
  }
  epilogue<VERIFY>(st, rsrc, voff, nmain * 2u * L, len, lane, nvalid, chunk0, digests, expected, ok);
}

// LDS-staged variant: the wave's 64 chunks are fetched COALESCED -- each
// 16-byte load instruction moves 8 whole 128-byte lines (8 lanes per chunk
// line) straight into LDS (buffer_load ... lds, no VGPR round trip) -- and
// each lane then reads its own chunk's line back with ds_read_b128.  Same
// bytes and VALU work as k_sha1_fixed, but the texture path handles 8 lines
// per instruction instead of 64 (one per lane).  Per wave one 8 KiB slot
// (64 rows x 128 B): slot s+1 is DMA'd while slot s (already in VGPRs) is
// compressed.  Within a row the 16-byte pieces are rotated by (row/2) mod 8
// so the 16 lanes of each ds_read_b128 pass hit distinct banks.
//
// The DMA is inline asm (hipcc neither orders builtin LDS-DMA against later
// ds_reads of the same bytes nor counts it), so the waits are explicit:
// vmcnt(0) before reading a slot, lgkmcnt(0) before overwriting it.
typedef int i32x4 __attribute__((ext_vector_type(4)));

#define BT_GLDS_ASM(POL)                                                                                \
  asm volatile("s_waitcnt lgkmcnt(0)\n\t"                                                              \
               "s_mov_b32 %0, m0\n\t"                                                                   \
               "s_mov_b32 m0, %10\n\t"                                                                  \
               "s_nop 0\n\t"                                                                            \
               "buffer_load_dwordx4 %1, %9, %11 offen" POL " lds\n\t"                                   \
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"                                                 \
               "buffer_load_dwordx4 %2, %9, %11 offen" POL " lds\n\t"                                   \
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"                                                 \
               "buffer_load_dwordx4 %3, %9, %11 offen" POL " lds\n\t"                                   \
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"                                                 \
               "buffer_load_dwordx4 %4, %9, %11 offen" POL " lds\n\t"                                   \
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"                                                 \
               "buffer_load_dwordx4 %5, %9, %11 offen" POL " lds\n\t"                                   \
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"                                                 \
               "buffer_load_dwordx4 %6, %9, %11 offen" POL " lds\n\t"                                   \
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"                                                 \
               "buffer_load_dwordx4 %7, %9, %11 offen" POL " lds\n\t"                                   \
               "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"                                                 \
               "buffer_load_dwordx4 %8, %9, %11 offen" POL " lds\n\t"                                   \
               "s_mov_b32 m0, %0"                                                                        \
               : "=&s"(keep)                                                                             \
               : "v"(voff[0]), "v"(voff[1]), "v"(voff[2]), "v"(voff[3]), "v"(voff[4]), "v"(voff[5]),     \
                 "v"(voff[6]), "v"(voff[7]), "s"(rsrc), "s"(lds), "s"(soff)                              \
               : "memory", "scc")

// Eight DMA loads = one 8 KiB slot (64 rows x 128 B) at LDS byte address lds;
// AUX 2 = non-temporal.  Waits for the wave's earlier ds_reads first (WAR).
template <int AUX>
__device__ __forceinline__ void glds_slot(const i32x4 rsrc, const uint32_t (&voff)[8], uint32_t soff, uint32_t lds) {
  uint32_t keep;
  if constexpr (AUX == 2)
    BT_GLDS_ASM(" nt");  // "offen nt lds"
  else
    BT_GLDS_ASM("");
}
#undef BT_GLDS_ASM

template <int AUX, bool VERIFY>
__global__ __launch_bounds__(kBlock, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_sha1_lds(
    const uint8_t *__restrict__ base, uint64_t n_chunks, uint32_t pitch, uint32_t len, uint8_t *__restrict__ digests,
    const uint8_t *__restrict__ expected, uint8_t *__restrict__ ok) {
  __shared__ u32x4 stage[kBlock / 64][64][8];  // [wave][row = chunk][16-byte piece, rotated]
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t chunk0 = (uint64_t)blockIdx.x * blockDim.x + (uint64_t)wave * 64u;
  if (chunk0 >= n_chunks) return;
  const uint64_t left = n_chunks - chunk0;
  const uint32_t nvalid = left < 64 ? (uint32_t)left : 64u;
  const uint32_t mine = lane < nvalid ? lane : nvalid - 1u;
  const uint32_t voff = mine * pitch;
  const uint32_t nrec = (nvalid - 1u) * pitch + ((len + 3u) & ~3u);
  uint8_t *wbase = (uint8_t *)(base + chunk0 * (uint64_t)pitch);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(wbase, (short)0, (int)nrec, 0x00020000);
  const uint64_t wb = (uint64_t)(uintptr_t)wbase;
  const i32x4 rsrc4 = {(int)__builtin_amdgcn_readfirstlane((uint32_t)wb),
                       (int)__builtin_amdgcn_readfirstlane((uint32_t)(wb >> 32) & 0xFFFFu),
                       (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000};

  // DMA instruction j, lane l: row q = 8j + l/8 (chunk min(q, nvalid-1)),
  // position l%8 holds piece (l%8 + q/2) % 8 of the row's 128-byte line.
  uint32_t dma_off[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t q = 8u * j + (lane >> 3);
    const uint32_t src = q < nvalid ? q : nvalid - 1u;
    dma_off[j] = src * pitch + (((lane & 7u) + (q >> 1)) & 7u) * 16u;
  }
  const uint32_t lds_wave = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)&stage[wave][0][0];
  // Lane c reads piece p of row c at position (p - c/2) % 8.
  const u32x4 *row = &stage[wave][lane][0];
  const uint32_t rot = lane >> 1;

  State st;
  st.init();
  const uint32_t nslots = (len >> 6) / 2u;  // 128-byte slots
  if (nslots) {
    glds_slot<AUX>(rsrc4, dma_off, 0u, lds_wave);
    for (uint32_t s = 0; s < nslots; ++s) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u32x4 q[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) q[p] = row[(p - rot) & 7u];
      if (s + 1 < nslots) glds_slot<AUX>(rsrc4, dma_off, (s + 1) * 128u, lds_wave);  // waits lgkmcnt(0) first
      __builtin_amdgcn_sched_barrier(0);
      compress_slot<1>(st, q);
    }
  }
  epilogue<VERIFY>(st, rsrc, voff, nslots * 2u, len, lane, nvalid, chunk0, digests, expected, ok);
}

// ---------------------------------------------------------------------------
// Latency kernel: small batches, where a chunk's latency is its serial chain.
// ---------------------------------------------------------------------------
// Below one wave per SIMD most SIMDs idle, and a lone wave issues at most one
// instruction per ~4 cycles (tools/latency_bench.py), so a chain costs its
// instruction count (8193 x 597 -> ~9 ms per 512 KiB).  Here every 64 chunks
// get a workgroup of two waves on two SIMDs of one CU:
//   wave S loads the message, byte-swaps, expands the schedule and adds K
//          (sha.c:186-200 and the K of DO_ROUND, sha.c:57-69), writing W+K
//          for 40 rounds at a time into an LDS slot, then the MD padding
//          block(s) (sha.c:536-543);
//   wave R runs the rounds from LDS and owns the state: 5 VALU per round
//          (f, two rotations, add3, add) + 20 ds_read_b128 per block.
// Two 20 KiB slots of one block each, one s_barrier per block: S fills slot
// b&1 while R consumes slot (b-1)&1.  Same arithmetic as compress(); only the
// work split differs.  Like k_sha1_fixed it takes an optional shorter tail
// chunk.
template <int T>
__device__ __forceinline__ constexpr uint32_t kconst() {
  return T < 20 ? 0x5a827999u : T < 40 ? 0x6ed9eba1u : T < 60 ? 0x8f1bbcdcu : 0xca62c1d6u;  // sha.c:66-69
}

template <int T>
__device__ __forceinline__ void round_wk(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                         uint32_t wk) {
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

// Rounds T..TEND-1 from a block's slot (4 W+K words per 16-byte LDS entry,
// lane-major).
template <int T, int TEND>
__device__ __forceinline__ void consume_wk(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                           const u32x4 *slot, uint32_t lane) {
  if constexpr (T < TEND) {
    const u32x4 q = slot[(T / 4) * 64 + lane];
    round_wk<T>(a, b, c, d, e, q.x);
    round_wk<T + 1>(a, b, c, d, e, q.y);
    round_wk<T + 2>(a, b, c, d, e, q.z);
    round_wk<T + 3>(a, b, c, d, e, q.w);
    consume_wk<T + 4, TEND>(a, b, c, d, e, slot, lane);
  }
}

// W+K of rounds T..TEND-1 into an LDS slot: 16-byte entry (T/4) of lane's
// block at slot[(T/4)*QS + lane*LS].  k_sha1_lat: QS = 64, LS = 1 (word-major,
// one chunk per lane); k_sha1_chain: QS = 1, LS = kChainStride (block-major).
template <int T, int TEND, int QS = 64, int LS = 1>
__device__ __forceinline__ void produce_wk(uint32_t (&w)[16], u32x4 *slot, uint32_t lane) {
  if constexpr (T < TEND) {
    u32x4 q;
    q.x = sched<T>(w) + kconst<T>();
    q.y = sched<T + 1>(w) + kconst<T + 1>();
    q.z = sched<T + 2>(w) + kconst<T + 2>();
    q.w = sched<T + 3>(w) + kconst<T + 3>();
    slot[(T / 4) * QS + lane * LS] = q;
    produce_wk<T + 4, TEND, QS, LS>(w, slot, lane);
  }
}

// Barrier accounting of k_sha1_lat.  S and R run different code, so the
// workgroup barrier is met from different call sites; s_barrier counts WAVES,
// and the kernel is correct only while both waves execute exactly the same
// number of barriers: nb_total + SLOTS - 1 each (S: one per produced block +
// SLOTS - 1 final; R: SLOTS - 1 before its loop + one per consumed block).  Any
// edit that changes one side's block count pairs the waves' barriers wrongly
// (S then overwrites a slot R is still reading) or leaves a wave waiting.
// Build with -DBT_SHA1_DEBUG_BARRIERS (`make dbgbar`) to count them per wave:
// every wave adds one check, its barrier count and, on a mismatch, one miss
// to g_bar_stats (vector atomics, lane 0), which bt_sha1_debug_barrier_stats
// reads back -- tests/test_gpu_barriers.py asserts zero misses AND the exact
// total the invariant predicts for each launch shape.
#ifdef BT_SHA1_DEBUG_BARRIERS
__device__ unsigned long long g_bar_stats[3];  // {waves checked, barriers counted, mismatches}
#define BT_LAT_BARRIER(cnt) \
  do {                      \
    ++(cnt);                \
    __syncthreads();        \
  } while (0)
#define BT_LAT_CHECK(cnt, want)                                              \
  do {                                                                       \
    if ((threadIdx.x & 63u) == 0) {                                          \
      atomicAdd(&g_bar_stats[0], 1ull);                                      \
      atomicAdd(&g_bar_stats[1], (unsigned long long)(cnt));                 \
      if ((uint64_t)(cnt) != (uint64_t)(want)) atomicAdd(&g_bar_stats[2], 1ull); \
    }                                                                        \
  } while (0)
#else
#define BT_LAT_BARRIER(cnt) __syncthreads()
#define BT_LAT_CHECK(cnt, want) ((void)0)
#endif

// One block through S into slot p of SLOTS, then the block's barrier.
template <int SLOTS>
__device__ __forceinline__ void produce_block(uint32_t (&w)[16], u32x4 (*lds)[20 * 64], uint32_t &p, uint32_t lane,
                                              uint32_t &nbar) {
  produce_wk<0, 80>(w, lds[p], lane);
  p = p + 1u == (uint32_t)SLOTS ? 0u : p + 1u;
  BT_LAT_BARRIER(nbar);
}

template <int T>
__device__ __forceinline__ void rounds_wk_regs(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                               const u32x4 (&q)[20]) {
  if constexpr (T < 80) {
    const u32x4 v = q[T / 4];
    round_wk<T>(a, b, c, d, e, v.x);
    round_wk<T + 1>(a, b, c, d, e, v.y);
    round_wk<T + 2>(a, b, c, d, e, v.z);
    round_wk<T + 3>(a, b, c, d, e, v.w);
    rounds_wk_regs<T + 4>(a, b, c, d, e, q);
  }
}

// R of k_sha1_lat<.., 3>: one block's 80 W+K words of this lane's chunk from a
// slot (lane-major 16-byte entries), and the 80 rounds on them.
__device__ __forceinline__ void lat_fetch(u32x4 (&q)[20], const u32x4 *slot, uint32_t lane) {
#pragma unroll
  for (int j = 0; j < 20; ++j) q[j] = slot[j * 64 + lane];
}

__device__ __forceinline__ void lat_rounds(State &st, const u32x4 (&q)[20]) {
  uint32_t a = st.h0, b = st.h1, c = st.h2, d = st.h3, e = st.h4;
  rounds_wk_regs<0>(a, b, c, d, e, q);
  st.h0 += a;  // sha.c:446-450
  st.h1 += b;
  st.h2 += c;
  st.h3 += d;
  st.h4 += e;
}

// SLOTS = 2: S one block ahead (40 KiB of LDS) -- the fastest form while
// each CU holds one workgroup.  SLOTS = 3: S two blocks ahead and R reading
// the next block into registers during the current one (60 KiB, so at most
// two workgroups per CU): it keeps the latency when two workgroups share a
// CU and their waves share SIMDs (32768 chunks: 6.8 ms vs 11.3 ms).
// MID: one COLUMN of each chunk -- len bytes (a 64-byte multiple) at `pitch`
// from the previous chunk's column -- for the host pipeline's column-split
// last batch (bt_sha1_api.cpp, chunks_host_on), each chunk's chaining state
// carried between launches in `state` (word k of chunk i at state[k*n_chunks
// + i]; SHA1Context.hash, sha.c:446-450):
//   kLatWhole  (0): whole chunks: IV, blocks, MD padding, digest;
//   kLatFirst  (1): IV, the column's blocks, state out;
//   kLatMiddle (2): state in, the column's blocks, state out;
//   kLatLast   (3): state in, the column's blocks, then the MD padding of a
//                   msg_len-byte message (sha.c:529-543), digest out.
constexpr int kLatWhole = 0, kLatFirst = 1, kLatMiddle = 2, kLatLast = 3;
template <bool VERIFY, int SLOTS = 2, int MID = kLatWhole>
__global__ __launch_bounds__(128) void k_sha1_lat(const uint8_t *__restrict__ base, uint64_t n_chunks, uint32_t pitch,
                                                  uint32_t len, uint8_t *__restrict__ digests,
                                                  const uint8_t *__restrict__ expected, uint8_t *__restrict__ ok,
                                                  uint32_t tail_len, uint32_t *__restrict__ state, uint64_t msg_len) {
  constexpr bool kPad = MID == kLatWhole || MID == kLatLast;  // ends with the MD padding + digest
  __shared__ u32x4 lds[SLOTS][20 * 64];  // SLOTS x 80 words x 64 lanes = SLOTS x 20 KiB
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint64_t chunk0 = (uint64_t)blockIdx.x * 64u;  // workgroup-uniform: both waves agree
  uint32_t nvalid;
  if (chunk0 < n_chunks) {
    const uint64_t left = n_chunks - chunk0;
    nvalid = left < 64 ? (uint32_t)left : 64u;
  } else {
    if (tail_len == 0 || chunk0 != ((n_chunks + 63u) & ~(uint64_t)63u)) return;
    chunk0 = n_chunks;
    nvalid = 1;
    len = tail_len;
  }
  const uint32_t nblocks = len >> 6, r = len & 63u;
  // + MD padding block(s).  Both waves execute nb_total + SLOTS - 1 barriers
  // (see "Barrier accounting" above).
  const uint32_t nb_total = kPad ? nblocks + (r >= 56u ? 2u : 1u) : nblocks;
  uint32_t nbar = 0;
  (void)nbar;
  if (wave == 0) {
    // ---- S: loads, schedule + K --------------------------------------------
    const uint32_t mine = lane < nvalid ? lane : nvalid - 1u;
    const uint32_t voff = mine * pitch;
    const uint32_t nrec = (nvalid - 1u) * pitch + ((len + 3u) & ~3u);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(base + chunk0 * (uint64_t)pitch), (short)0, (int)nrec, 0x00020000);
    // Four-block register ring, three blocks of prefetch (~2.5 us at R's
    // pace): S must never stall on memory, or R waits at the barrier.  Loads
    // past nrec are range-checked zeros, so they need no guard (and no branch
    // that would make the compiler wait for them, see absorb_ring).
    uint32_t slot = 0;  // LDS slot the next block goes to
    u32x4 ring[4][4];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) ring[k][i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, k * 64u + 16u * i, 0);
    for (uint32_t b = 0; b < nblocks; b += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          ring[(k + 3) % 4][i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, (b + k + 3) * 64u + 16u * i, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (b + k < nblocks) {  // wave-uniform
          uint32_t w[16];
          block_from_le(w, ring[k][0], ring[k][1], ring[k][2], ring[k][3]);
          produce_block<SLOTS>(w, lds, slot, lane, nbar);
        }
      }
    }
    if constexpr (kPad) {
      // Tail bytes + MD padding (sha.c:536-543), as finish() lays them out.
      uint32_t tail[16];
      load_tail(tail, rsrc, voff, nblocks, r);
      const uint32_t wi = r >> 2, mark = 0x80000000u >> ((r & 3) * 8);
#pragma unroll
      for (int j = 0; j < 16; ++j) tail[j] |= (j == (int)wi) ? mark : 0u;
      const uint64_t bits = (MID == kLatLast ? msg_len : (uint64_t)len) * 8ull;
      if (r >= 56u) {
        produce_block<SLOTS>(tail, lds, slot, lane, nbar);
#pragma unroll
        for (int j = 0; j < 16; ++j) tail[j] = 0u;
      }
      tail[14] = (uint32_t)(bits >> 32);
      tail[15] = (uint32_t)bits;
      produce_block<SLOTS>(tail, lds, slot, lane, nbar);
    }
#pragma unroll
    for (int k = 0; k < SLOTS - 1; ++k) BT_LAT_BARRIER(nbar);  // pair with R's last barriers
    BT_LAT_CHECK(nbar, nb_total + SLOTS - 1u);
  } else {
    // ---- R: rounds -----------------------------------------------------------
    const uint64_t mine = chunk0 + (lane < nvalid ? lane : nvalid - 1u);
    State st;
    if constexpr (MID == kLatMiddle || MID == kLatLast) {
      st.h0 = state[mine];
      st.h1 = state[n_chunks + mine];
      st.h2 = state[2 * n_chunks + mine];
      st.h3 = state[3 * n_chunks + mine];
      st.h4 = state[4 * n_chunks + mine];
    } else {
      st.init();
    }
    if constexpr (SLOTS == 2) {
      BT_LAT_BARRIER(nbar);  // block 0 is in slot 0
      for (uint32_t b = 0; b < nb_total; ++b) {
        uint32_t a = st.h0, bb = st.h1, c = st.h2, d = st.h3, e = st.h4;
        consume_wk<0, 80>(a, bb, c, d, e, lds[b & 1u], lane);
        BT_LAT_BARRIER(nbar);
        st.h0 += a;  // sha.c:446-450
        st.h1 += bb;
        st.h2 += c;
        st.h3 += d;
        st.h4 += e;
      }
    } else {
      // S runs two blocks ahead: once barrier b+2 has passed, blocks b and
      // b+1 are both in LDS, so R reads block b+1 into registers while block
      // b's rounds run.  S overwrites slot (b+2) % 3 = (b-1) % 3 only after
      // barrier b+2, by which R has consumed block b-1 (its reads completed
      // before barrier b+1, which waits for them).
      BT_LAT_BARRIER(nbar);  // block 0 is in
      BT_LAT_BARRIER(nbar);  // block 1 (or S's first closing barrier) is in
      u32x4 wa[20], wb[20];
      lat_fetch(wa, lds[0], lane);
      uint32_t sb = 0;  // slot of block b
      for (uint32_t b = 0; b < nb_total; b += 2) {
        const uint32_t s1 = sb + 1u == 3u ? 0u : sb + 1u;
        const uint32_t s2 = s1 + 1u == 3u ? 0u : s1 + 1u;
        lat_fetch(wb, lds[b + 1 < nb_total ? s1 : sb], lane);
        lat_rounds(st, wa);
        BT_LAT_BARRIER(nbar);  // block b + 2 is in
        if (b + 1 < nb_total) {  // wave-uniform
          lat_fetch(wa, lds[b + 2 < nb_total ? s2 : s1], lane);
          lat_rounds(st, wb);
          BT_LAT_BARRIER(nbar);  // block b + 3 is in
        }
        sb = s2;
      }
    }
    BT_LAT_CHECK(nbar, nb_total + SLOTS - 1u);
    if constexpr (kPad) {
      store_digest<VERIFY>(st, lane, nvalid, chunk0, digests, expected, ok);
    } else if (lane < nvalid) {
      state[mine] = st.h0;
      state[n_chunks + mine] = st.h1;
      state[2 * n_chunks + mine] = st.h2;
      state[3 * n_chunks + mine] = st.h3;
      state[4 * n_chunks + mine] = st.h4;
    }
  }
}

// ---------------------------------------------------------------------------
// Chain kernel: ONE message per workgroup, for callers that wait on a single
// serial chain (shahash, SHA1Update / SHA1Final, a handful of ragged
// messages).  Same S / R split as k_sha1_lat, but S works across BLOCKS of
// the one message instead of across chunks: lane j of S byte-swaps block
// b0+j, expands its schedule and adds K (sha.c:186-200, 57-69) -- 64 blocks
// at once -- and R runs the rounds of those 64 blocks back to back from LDS
// (broadcast ds_read_b128, 5 VALU per round).  One barrier per 64 blocks
// instead of one per block, and S is never on R's critical path (it finishes
// a batch in a few microseconds; R takes ~50).  S reads the message wherever
// it is -- device memory, or pinned host memory directly over PCIe, so the
// drop-in calls need no H2D copy -- and builds the MD padding block(s)
// itself (sha.c:529-543).
//   MID = true : SHA1Update/SHA1Final midstate -- state[5] (SHA1Context.hash
//                order) advanced over fixed_len/64 whole blocks of `base`.
//   MID = false: message i = base + (offsets ? offsets[i] : i*pitch), length
//                lens ? lens[i] : fixed_len, digest i (big-endian, any
//                alignment) to digests + 20*i.  blockIdx.x = message.
// Barrier accounting as in k_sha1_lat: both waves execute nbatch + 1.
// ---------------------------------------------------------------------------
constexpr uint32_t kChainBatch = 64;  // blocks per LDS slot = lanes of S

// Block g of a message (nfull whole blocks, r tail bytes, bits total length)
// as 16 big-endian words: message block, tail block or length-only block.
template <bool MID>
__device__ __forceinline__ void chain_block(uint32_t (&w)[16], const uint8_t *p, uint64_t g, uint64_t nfull, uint32_t r,
                                            uint64_t bits) {
  if (g < nfull) {
    u32x4 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) __builtin_memcpy(&q[i], p + 64 * g + 16 * i, 16);  // any alignment
    block_from_le(w, q[0], q[1], q[2], q[3]);
    return;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = 0u;
  if constexpr (!MID) {
    if (g == nfull) {  // tail bytes + 0x80 (+ the length when r <= 55)
      const uint8_t *t = p + 64 * nfull;
      for (uint32_t k = 0; k < r; ++k) w[k >> 2] |= (uint32_t)t[k] << (24 - 8 * (k & 3));
      w[r >> 2] |= 0x80000000u >> ((r & 3) * 8);
      if (r < 56) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
      }
    } else {  // r >= 56: a length-only block follows
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
  }
}

// R side of the chain kernel.  A slot holds 64 blocks block-major: block k's
// 80 W+K words are 20 16-byte entries at slot[k*kChainStride ..] (stride 21:
// S's 64 lanes then write to spread banks).  R needs one word per round, and
// its 64 lanes all run the same chain, so instead of broadcasting every word
// to every lane (20 ds_read_b128 per block) lane L < 16 reads words 4L..4L+3
// and lane L < 4 words 64+4L..64+4L+3 -- two ds_read_b128 per block -- and
// round t takes its word from lane t/4 through a DPP row shift folded into
// the round's add (v_add_u32_dpp ... row_shl:t/4).  Lane 0 therefore runs
// the exact chain (sha.c:57-64) and owns the result; the other lanes compute
// garbage.  tools/ubench/chain_floor: 5.99 ms per 512 KiB chain against 6.26
// for the broadcast form and 5.65 for the same rounds with no loads at all.
constexpr uint32_t kChainStride = 21;

template <int T>
__device__ __forceinline__ uint32_t wk_from_lane(const u32x4 &A, const u32x4 &B) {
  constexpr int g = T < 64 ? T / 4 : (T - 64) / 4;
  const uint32_t src = T < 64 ? A[T % 4] : B[T % 4];
  if constexpr (g == 0) return src;
  else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)src, 0x100 + g, 0xF, 0xF, false);  // row_shl:g
}

template <int T>
__device__ __forceinline__ void chain_rounds_from(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                                  const u32x4 &A, const u32x4 &B) {
  if constexpr (T < 80) {
    round_wk<T>(a, b, c, d, e, wk_from_lane<T>(A, B));
    chain_rounds_from<T + 1>(a, b, c, d, e, A, B);
  }
}

__device__ __forceinline__ void chain_rounds(State &st, const u32x4 &A, const u32x4 &B) {
  uint32_t a = st.h0, b = st.h1, c = st.h2, d = st.h3, e = st.h4;
  chain_rounds_from<0>(a, b, c, d, e, A, B);
  st.h0 += a;  // sha.c:446-450
  st.h1 += b;
  st.h2 += c;
  st.h3 += d;
  st.h4 += e;
}

template <bool MID, bool VERIFY = false>
__global__ __launch_bounds__(128) void k_sha1_chain(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offsets,
                                                    const uint32_t *__restrict__ lens, uint64_t pitch, uint64_t fixed_len,
                                                    uint64_t tail_len, uint32_t *__restrict__ state,
                                                    uint8_t *__restrict__ digests, const uint8_t *__restrict__ expected,
                                                    uint8_t *__restrict__ ok, uint32_t *__restrict__ done,
                                                    uint32_t seq) {
  __shared__ u32x4 lds[2][kChainStride * kChainBatch];  // 2 slots x 64 blocks x (80 + 4) words = 42 KiB
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t i = blockIdx.x;
  const uint8_t *p = base + (offsets ? offsets[i] : i * pitch);
  // tail_len != 0: the last message is a shorter one (make_chunks' last fread).
  const uint64_t len = lens ? (uint64_t)lens[i] : (tail_len && i + 1 == gridDim.x ? tail_len : fixed_len);
  const uint64_t nfull = len >> 6;
  const uint32_t r = (uint32_t)(len & 63u);
  const uint64_t nb_total = MID ? nfull : nfull + (r >= 56u ? 2u : 1u);
  const uint64_t nbatch = (nb_total + kChainBatch - 1) / kChainBatch;
  uint32_t nbar = 0;
  (void)nbar;
  if (wave == 0) {
    // ---- S: lane j prepares block b0 + j ----------------------------------
    for (uint64_t bt = 0; bt < nbatch; ++bt) {
      const uint64_t g = bt * kChainBatch + lane;
      uint32_t w[16];
      chain_block<MID>(w, p, g < nb_total ? g : nb_total, nfull, r, len * 8ull);
      produce_wk<0, 80, 1, kChainStride>(w, lds[bt & 1u], lane);
      BT_LAT_BARRIER(nbar);
    }
    BT_LAT_BARRIER(nbar);  // pairs with R's last barrier
    BT_LAT_CHECK(nbar, nbatch + 1u);
  } else {
    // ---- R: the chain --------------------------------------------------------
    State st;
    if constexpr (MID) {
      st.h0 = state[0]; st.h1 = state[1]; st.h2 = state[2]; st.h3 = state[3]; st.h4 = state[4];
    } else {
      st.init();
    }
    BT_LAT_BARRIER(nbar);  // batch 0 is in slot 0
    const uint32_t l16 = lane & 15u, l4 = lane & 3u;
    for (uint64_t bt = 0; bt < nbatch; ++bt) {
      const u32x4 *slot = lds[bt & 1u];
      const uint64_t left = nb_total - bt * kChainBatch;
      const uint32_t nb = left < kChainBatch ? (uint32_t)left : kChainBatch;
      // Block k+1's two reads are issued before block k's rounds.
      u32x4 A = slot[l16], B = slot[16 + l4];
      for (uint32_t k = 0; k < nb; ++k) {
        const u32x4 *nxt = slot + (k + 1 < nb ? k + 1 : k) * kChainStride;
        const u32x4 An = nxt[l16], Bn = nxt[16 + l4];
        chain_rounds(st, A, B);
        A = An;
        B = Bn;
      }
      BT_LAT_BARRIER(nbar);
    }
    BT_LAT_CHECK(nbar, nbatch + 1u);
    if (lane == 0) {
      if constexpr (MID) {
        state[0] = st.h0; state[1] = st.h1; state[2] = st.h2; state[3] = st.h3; state[4] = st.h4;
      } else {
        const uint32_t h[5] = {st.h0, st.h1, st.h2, st.h3, st.h4};
        if (digests) {
          uint8_t *o = digests + 20 * i;
#pragma unroll
          for (int k = 0; k < 5; ++k) {  // sha.c:550-553
            o[4 * k] = (uint8_t)(h[k] >> 24);
            o[4 * k + 1] = (uint8_t)(h[k] >> 16);
            o[4 * k + 2] = (uint8_t)(h[k] >> 8);
            o[4 * k + 3] = (uint8_t)h[k];
          }
        }
        if constexpr (VERIFY) {  // memcmp(hash, chunk->hash, 20) == 0, util.c:313
          const uint8_t *x = expected + 20 * i;
          uint32_t diff = 0;
#pragma unroll
          for (int k = 0; k < 20; ++k) diff |= (uint32_t)x[k] ^ ((h[k >> 2] >> (24 - 8 * (k & 3))) & 0xFFu);
          ok[i] = diff == 0;
        }
      }
      // Completion word for a host that spins instead of waiting on the
      // stream (drop-in calls): released at system scope after the results.
      if (done) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// Latency kernel for RAGGED batches (bt_sha1_ragged_dev with 2 x CUs < n <=
// 128 x CUs messages): k_sha1_lat's loader / round-wave split with per-lane
// message pointers and lengths.  Lane j of both waves owns message 64*wg + j;
// the waves run to the longest message of the 64, lane j latches its state
// after its own last block.  S reads any alignment (16-byte loads as in
// SrcBytes) through a four-block register ring; lanes whose message has no
// whole block read a static zero block instead of running past their message.
// ---------------------------------------------------------------------------
__device__ u32x4 kZeroBlock[4];

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

template <int SLOTS>
__global__ __launch_bounds__(128) void k_sha1_lat_ragged(const uint8_t *__restrict__ base,
                                                         const uint64_t *__restrict__ offsets,
                                                         const uint32_t *__restrict__ lens, uint64_t pitch,
                                                         uint32_t fixed_len, uint64_t n, uint8_t *__restrict__ digests) {
  __shared__ u32x4 lds[SLOTS][20 * 64];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t idx = (uint64_t)blockIdx.x * 64u + lane;
  const uint64_t mi = idx < n ? idx : n - 1;  // lanes past the end re-hash the last message, no store
  const uint8_t *p = base + (offsets ? offsets[mi] : mi * pitch);
  const uint32_t len = lens ? lens[mi] : fixed_len;
  const uint32_t nfull = len >> 6, r = len & 63u;
  const uint32_t nb = nfull + (r >= 56u ? 2u : 1u);
  // Both waves hold the same per-lane lengths, so they agree on the trip count
  // and on the barrier count: nbmax + SLOTS - 1 each.
  const uint32_t nbmax = __builtin_amdgcn_readfirstlane(wave_max(nb));
  uint32_t nbar = 0;
  (void)nbar;
  if (wave == 0) {
    // ---- S -------------------------------------------------------------------
    const uint8_t *lp = nfull ? p : (const uint8_t *)kZeroBlock;
    const uint32_t lmax = nfull ? nfull - 1u : 0u;
    const uint64_t bits = (uint64_t)len * 8ull;
    // The tail bytes + 0x80 (sha.c:536-538) are read once, up front: a load in
    // the per-block lane-divergent branch below would make the compiler wait
    // for the whole prefetch ring at the branch join on every block.
    uint32_t tw[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) tw[j] = 0u;
    {
      const uint8_t *t = p + 64u * nfull;
      for (uint32_t q = 0; q < r; ++q) tw[q >> 2] |= (uint32_t)t[q] << (24 - 8 * (q & 3));
      tw[r >> 2] |= 0x80000000u >> ((r & 3) * 8);
    }
    uint32_t slot = 0;
    u32x4 ring[4][4];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) __builtin_memcpy(&ring[k][i], lp + 64u * ((uint32_t)k < lmax ? k : lmax) + 16 * i, 16);
    for (uint32_t b = 0; b < nbmax; b += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t nx = b + k + 3u;
#pragma unroll
        for (int i = 0; i < 4; ++i) __builtin_memcpy(&ring[(k + 3) % 4][i], lp + 64u * (nx < lmax ? nx : lmax) + 16 * i, 16);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t bk = b + k;
        if (bk < nbmax) {  // wave-uniform
          uint32_t w[16];
          if (bk < nfull) {
            block_from_le(w, ring[k][0], ring[k][1], ring[k][2], ring[k][3]);
          } else {  // the tail block, then (r >= 56) a length-only block, sha.c:536-543
#pragma unroll
            for (int j = 0; j < 16; ++j) w[j] = bk == nfull ? tw[j] : 0u;
            if ((bk == nfull && r < 56u) || bk == nfull + 1u) {
              w[14] = (uint32_t)(bits >> 32);
              w[15] = (uint32_t)bits;
            }
          }
          produce_block<SLOTS>(w, lds, slot, lane, nbar);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < SLOTS - 1; ++k) BT_LAT_BARRIER(nbar);  // pair with R's last barriers
    BT_LAT_CHECK(nbar, nbmax + SLOTS - 1u);
  } else {
    // ---- R -------------------------------------------------------------------
    State st, fin;
    st.init();
    fin = st;
    auto latch = [&](uint32_t b) {  // this lane's last block done: keep its state
      if (b + 1u == nb) fin = st;
    };
    if constexpr (SLOTS == 2) {
      BT_LAT_BARRIER(nbar);
      for (uint32_t b = 0; b < nbmax; ++b) {
        uint32_t a = st.h0, bb = st.h1, c = st.h2, d = st.h3, e = st.h4;
        consume_wk<0, 80>(a, bb, c, d, e, lds[b & 1u], lane);
        BT_LAT_BARRIER(nbar);
        st.h0 += a;  // sha.c:446-450
        st.h1 += bb;
        st.h2 += c;
        st.h3 += d;
        st.h4 += e;
        latch(b);
      }
    } else {
      BT_LAT_BARRIER(nbar);
      BT_LAT_BARRIER(nbar);
      u32x4 wa[20], wb[20];
      lat_fetch(wa, lds[0], lane);
      uint32_t sb = 0;
      for (uint32_t b = 0; b < nbmax; b += 2) {
        const uint32_t s1 = sb + 1u == 3u ? 0u : sb + 1u;
        const uint32_t s2 = s1 + 1u == 3u ? 0u : s1 + 1u;
        lat_fetch(wb, lds[b + 1 < nbmax ? s1 : sb], lane);
        lat_rounds(st, wa);
        latch(b);
        BT_LAT_BARRIER(nbar);
        if (b + 1 < nbmax) {
          lat_fetch(wa, lds[b + 2 < nbmax ? s2 : s1], lane);
          lat_rounds(st, wb);
          latch(b + 1);
          BT_LAT_BARRIER(nbar);
        }
        sb = s2;
      }
    }
    BT_LAT_CHECK(nbar, nbmax + SLOTS - 1u);
    if (idx < n) {
      uint8_t *o = digests + idx * 20u;
      const uint32_t h[5] = {fin.h0, fin.h1, fin.h2, fin.h3, fin.h4};
#pragma unroll
      for (int k = 0; k < 5; ++k) {  // byte stores: digests need no alignment here
        o[4 * k] = (uint8_t)(h[k] >> 24);
        o[4 * k + 1] = (uint8_t)(h[k] >> 16);
        o[4 * k + 2] = (uint8_t)(h[k] >> 8);
        o[4 * k + 3] = (uint8_t)h[k];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Generic paths (64-bit addressing, any alignment).
// ---------------------------------------------------------------------------
// Block source for absorb_ring: how one 64-byte block is fetched into a
// register slot and turned into 16 big-endian words (sha.c:186-189).  The
// loads are 16-byte loads at the message's own alignment: gfx950 under HSA
// runs in unaligned-access mode (hipcc emits global_load_dwordx4 for an
// unaligned memcpy), so a byte-misaligned message costs four loads per block
// like an aligned one, instead of one load per byte or word.
struct SrcBytes {
  typedef u32x4 Slot[4];
  const uint8_t *p;
  __device__ __forceinline__ void load(Slot &s, uint64_t k) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) __builtin_memcpy(&s[i], p + 64 * k + 16 * i, 16);
  }
  __device__ __forceinline__ void words(uint32_t (&w)[16], const Slot &s) const { block_from_le(w, s[0], s[1], s[2], s[3]); }
};

// Whole blocks through a 3-slot register ring: block k+2 is fetched while
// block k is compressed, so a lone chain (shahash, a ragged message, the
// streaming API) does not wait on memory once per block.  Prefetch indices
// are clamped to the message's last block (re-read, never used) rather than
// branched around: a load inside a branch makes the compiler wait for every
// outstanding load at the join (vmcnt(0), seen in the ISA), which turns the
// ring back into one memory round trip per block.
template <class Src>
__device__ __forceinline__ void absorb_ring(State &st, const Src &src, uint64_t nblocks) {
  if (nblocks == 0) return;
  const uint64_t last = nblocks - 1;
  typename Src::Slot ring[3];
  src.load(ring[0], 0);
  src.load(ring[1], last < 1 ? last : 1);
  uint64_t k = 0;
  for (; k + 3 <= nblocks; k += 3) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const uint64_t nx = k + s + 2;
      src.load(ring[(s + 2) % 3], nx < last ? nx : last);
      __builtin_amdgcn_sched_barrier(0);
      uint32_t w[16];
      src.words(w, ring[s]);
      compress(st, w);
    }
  }
  // 0..2 blocks left; they are already in ring[0], ring[1].
  if (k < nblocks) {
    uint32_t w[16];
    src.words(w, ring[0]);
    compress(st, w);
  }
  if (k + 1 < nblocks) {
    uint32_t w[16];
    src.words(w, ring[1]);
    compress(st, w);
  }
}

__device__ __forceinline__ void absorb_blocks(State &st, const uint8_t *p, uint64_t nblocks) {
  absorb_ring(st, SrcBytes{p}, nblocks);
}

__device__ __forceinline__ void absorb_tail_and_finish(State &st, const uint8_t *p, uint32_t r, uint64_t len) {
  uint32_t tail[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if ((uint32_t)(4 * j + b) < r) v |= (uint32_t)p[4 * j + b] << (24 - 8 * b);
    tail[j] = v;
  }
  finish(st, tail, r, len);
}

// Message i = base[offsets[i] .. + lens[i]); with offsets == NULL the batch is
// strided instead: message i = base[i*pitch .. + fixed_len).
__global__ __launch_bounds__(kBlock) void k_sha1_ragged(const uint8_t *__restrict__ base,
                                                        const uint64_t *__restrict__ offsets,
                                                        const uint32_t *__restrict__ lens, uint64_t pitch,
                                                        uint32_t fixed_len, uint64_t n,
                                                        uint8_t *__restrict__ digests) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *p = base + (offsets ? offsets[i] : i * pitch);
  const uint32_t len = offsets ? lens[i] : fixed_len;
  State st;
  st.init();
  const uint64_t nb = len >> 6;
  absorb_blocks(st, p, nb);
  absorb_tail_and_finish(st, p + nb * 64u, len & 63u, len);
  uint8_t *o = digests + i * 20u;
  const uint32_t h[5] = {st.h0, st.h1, st.h2, st.h3, st.h4};
#pragma unroll
  for (int k = 0; k < 5; ++k) {  // byte stores: digests need no alignment here
    o[4 * k] = (uint8_t)(h[k] >> 24);
    o[4 * k + 1] = (uint8_t)(h[k] >> 16);
    o[4 * k + 2] = (uint8_t)(h[k] >> 8);
    o[4 * k + 3] = (uint8_t)h[k];
  }
}

// ---------------------------------------------------------------------------
// Frozen synthetic generator: word g of the stream = splitmix64(seed + g),
// stored little-endian (mirrored by oracle/sha1_oracle.c:or_fill_synthetic).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void k_fill_synthetic(uint8_t *__restrict__ buf, uint64_t nbytes,
                                                           uint64_t first_word, uint64_t seed) {
  const uint64_t nw = nbytes >> 3;
  const uint64_t npairs = nw >> 1;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t s0 = seed + first_word;
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  for (uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x; p < npairs; p += stride) {
    u64x2 v;
    v.x = splitmix64(s0 + 2 * p);
    v.y = splitmix64(s0 + 2 * p + 1);
    *(u64x2 *)(buf + 16 * p) = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    for (uint64_t g = npairs * 2; g * 8 < nbytes; ++g) {
      const uint64_t v = splitmix64(s0 + g);
      for (uint64_t b = 0; b < 8 && g * 8 + b < nbytes; ++b) buf[g * 8 + b] = (uint8_t)(v >> (8 * b));
    }
  }
}

// ---------------------------------------------------------------------------
// Digest lookup: get_chunk_id / find_chunk (util.c:3-39) for large tables.
// Open addressing over a power-of-two slot array of (index+1) u32 values,
// keyed by the digest's first 8 bytes (SHA-1 output is uniform); duplicates
// keep the smallest index, matching the reference's first-match scan.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_digest(const uint8_t *p, uint32_t (&d)[5]) {
  const uint32_t *q = (const uint32_t *)p;  // 20-byte records are 4-byte aligned
#pragma unroll
  for (int k = 0; k < 5; ++k) d[k] = q[k];
}

__device__ __forceinline__ bool same_digest(const uint32_t (&a)[5], const uint32_t (&b)[5]) {
  return ((a[0] ^ b[0]) | (a[1] ^ b[1]) | (a[2] ^ b[2]) | (a[3] ^ b[3]) | (a[4] ^ b[4])) == 0;
}

__global__ __launch_bounds__(kBlock) void k_lookup_build(const uint8_t *__restrict__ table, uint64_t n,
                                                         uint32_t *__restrict__ slots, uint32_t mask) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t key[5];
  load_digest(table + 20 * i, key);
  uint32_t s = key[0] & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe, s = (s + 1) & mask) {
    const uint32_t old = atomicCAS(&slots[s], 0u, (uint32_t)(i + 1));
    if (old == 0) return;
    uint32_t other[5];
    load_digest(table + 20 * (uint64_t)(old - 1), other);
    if (same_digest(key, other)) {
      atomicMin(&slots[s], (uint32_t)(i + 1));
      return;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_lookup_query(const uint8_t *__restrict__ table,
                                                         const uint32_t *__restrict__ slots, uint32_t mask,
                                                         const uint8_t *__restrict__ queries, uint64_t m,
                                                         int64_t *__restrict__ index) {
  const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q >= m) return;
  uint32_t key[5];
  load_digest(queries + 20 * q, key);
  uint32_t s = key[0] & mask;
  int64_t r = -1;
  for (uint32_t probe = 0; probe <= mask; ++probe, s = (s + 1) & mask) {
    const uint32_t v = slots[s];
    if (v == 0) break;
    uint32_t other[5];
    load_digest(table + 20 * (uint64_t)(v - 1), other);
    if (same_digest(key, other)) {
      r = (int64_t)v - 1;
      break;
    }
  }
  index[q] = r;
}

}  // namespace btsha1

// ---------------------------------------------------------------------------
// Launchers (C++ linkage, used by the C-ABI layer in bt_sha1_api.cpp).
// ---------------------------------------------------------------------------
using namespace btsha1;

// Compute units of the current device, cached per device id.
uint32_t btsha1_device_cus() {
  static uint32_t cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  uint32_t v = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
  if (!v) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    v = (uint32_t)cus;
    __atomic_store_n(&cache[dev], v, __ATOMIC_RELAXED);
  }
  return v;
}

// Below one wave per SIMD (CUs x 4 SIMDs x 64 lanes; 65536 chunks on a full
// MI355X) use one-wave workgroups so the dispatcher spreads the waves over
// distinct CUs instead of stacking four per CU: a chunk's latency is its
// serial 8193-block chain, so a lone wave per SIMD finishes the batch soonest.
static uint32_t chain_workgroup(uint64_t n) { return n < (uint64_t)btsha1_device_cus() * 4u * 64u ? 64u : (uint32_t)kBlock; }

template <int NBUF, int L, int AUX>
static hipError_t launch_fixed_v(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                                 const uint8_t *d_exp, uint8_t *d_ok, hipStream_t s, uint32_t tail_len,
                                 uint64_t *d_stamps = nullptr) {
  const uint32_t wg = chain_workgroup(n);
  const uint64_t threads = tail_len ? ((n + 63) & ~(uint64_t)63) + 64 : n;  // + the tail wave
  const uint64_t grid = (threads + wg - 1) / wg;
  if (d_stamps)
    hipLaunchKernelGGL((k_sha1_fixed<NBUF, L, AUX, false, true>), dim3((uint32_t)grid), dim3(wg), 0, s,
                       (const uint8_t *)d_in, n, pitch, len, d_dig, d_exp, d_ok, 0u, d_stamps);
  else if (d_ok)
    hipLaunchKernelGGL((k_sha1_fixed<NBUF, L, AUX, true>), dim3((uint32_t)grid), dim3(wg), 0, s,
                       (const uint8_t *)d_in, n, pitch, len, d_dig, d_exp, d_ok, tail_len, nullptr);
  else
    hipLaunchKernelGGL((k_sha1_fixed<NBUF, L, AUX, false>), dim3((uint32_t)grid), dim3(wg), 0, s,
                       (const uint8_t *)d_in, n, pitch, len, d_dig, d_exp, d_ok, tail_len, nullptr);
  return hipGetLastError();
}

template <int AUX>
static hipError_t launch_lds(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                             const uint8_t *d_exp, uint8_t *d_ok, hipStream_t s) {
  const uint64_t grid = (n + kBlock - 1) / kBlock;
  if (d_ok)
    hipLaunchKernelGGL((k_sha1_lds<AUX, true>), dim3((uint32_t)grid), dim3(kBlock), 0, s, (const uint8_t *)d_in, n, pitch,
                       len, d_dig, d_exp, d_ok);
  else
    hipLaunchKernelGGL((k_sha1_lds<AUX, false>), dim3((uint32_t)grid), dim3(kBlock), 0, s, (const uint8_t *)d_in, n, pitch,
                       len, d_dig, d_exp, d_ok);
  return hipGetLastError();
}
// Up to one workgroup per CU k_sha1_lat runs with two LDS slots; beyond that
// (two workgroups per CU, whose waves then share SIMDs) with three, where S
// is two blocks ahead and R never waits on it: 32768 chunks 6.8 ms against
// 11.3 ms for the two-slot form and 9.1 ms for the hot kernel.  The 60 KiB
// three-slot workgroup also caps a CU at two of them.
template <int SLOTS>
static hipError_t launch_lat_s(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                               const uint8_t *d_exp, uint8_t *d_ok, hipStream_t s, uint32_t tail_len, uint64_t grid) {
  if (d_ok)
    hipLaunchKernelGGL((k_sha1_lat<true, SLOTS>), dim3((uint32_t)grid), dim3(128), 0, s, (const uint8_t *)d_in, n,
                       pitch, len, d_dig, d_exp, d_ok, tail_len, nullptr, 0ull);
  else
    hipLaunchKernelGGL((k_sha1_lat<false, SLOTS>), dim3((uint32_t)grid), dim3(128), 0, s, (const uint8_t *)d_in, n,
                       pitch, len, d_dig, d_exp, d_ok, tail_len, nullptr, 0ull);
  return hipGetLastError();
}

template <int SLOTS, int MID, bool VERIFY = false>
static hipError_t launch_column_s(const void *d_col, uint64_t n, uint32_t pitch, uint32_t width, uint32_t *d_state,
                                  uint64_t msg_len, uint8_t *d_dig, const uint8_t *d_exp, uint8_t *d_ok, hipStream_t s,
                                  uint64_t grid) {
  hipLaunchKernelGGL((k_sha1_lat<VERIFY, SLOTS, MID>), dim3((uint32_t)grid), dim3(128), 0, s, (const uint8_t *)d_col, n,
                     pitch, width, d_dig, d_exp, d_ok, 0u, d_state, msg_len);
  return hipGetLastError();
}

template <int MID, bool VERIFY = false>
static hipError_t launch_column_m(const void *d_col, uint64_t n, uint32_t pitch, uint32_t width, uint32_t *d_state,
                                  uint64_t msg_len, uint8_t *d_dig, const uint8_t *d_exp, uint8_t *d_ok,
                                  hipStream_t s) {
  const uint64_t grid = (n + 63) / 64;
  return grid > btsha1_device_cus()
             ? launch_column_s<3, MID, VERIFY>(d_col, n, pitch, width, d_state, msg_len, d_dig, d_exp, d_ok, s, grid)
             : launch_column_s<2, MID, VERIFY>(d_col, n, pitch, width, d_state, msg_len, d_dig, d_exp, d_ok, s, grid);
}

hipError_t btsha1_launch_column(const void *d_col, uint64_t n, uint32_t pitch, uint32_t width, int part,
                                uint32_t *d_state, uint64_t msg_len, uint8_t *d_dig, hipStream_t s,
                                const uint8_t *d_exp, uint8_t *d_ok) {
  if (n == 0) return hipSuccess;
  if (!d_state || width == 0 || (width & 63u) || pitch < width || (pitch & 15u) || ((uintptr_t)d_col & 15u) ||
      64 * (uint64_t)pitch >= (1ull << 32) || (d_ok && (!d_exp || part != BTSHA1_COLUMN_LAST)))
    return hipErrorInvalidValue;
  switch (part) {
    case BTSHA1_COLUMN_FIRST:
      return launch_column_m<kLatFirst>(d_col, n, pitch, width, d_state, 0, nullptr, nullptr, nullptr, s);
    case BTSHA1_COLUMN_MIDDLE:
      return launch_column_m<kLatMiddle>(d_col, n, pitch, width, d_state, 0, nullptr, nullptr, nullptr, s);
    case BTSHA1_COLUMN_LAST:
      if ((!d_dig && !d_ok) || ((uintptr_t)d_dig & 3u)) return hipErrorInvalidValue;
      return d_ok ? launch_column_m<kLatLast, true>(d_col, n, pitch, width, d_state, msg_len, d_dig, d_exp, d_ok, s)
                  : launch_column_m<kLatLast>(d_col, n, pitch, width, d_state, msg_len, d_dig, nullptr, nullptr, s);
    default: return hipErrorInvalidValue;
  }
}

static hipError_t launch_lat(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                             const uint8_t *d_exp, uint8_t *d_ok, hipStream_t s, uint32_t tail_len) {
  const uint64_t grid = (n + 63) / 64 + (tail_len ? 1 : 0);
  return grid > btsha1_device_cus() ? launch_lat_s<3>(d_in, n, pitch, len, d_dig, d_exp, d_ok, s, tail_len, grid)
                                    : launch_lat_s<2>(d_in, n, pitch, len, d_dig, d_exp, d_ok, s, tail_len, grid);
}

// Batches of at most this many chunks take the latency kernel (0: never).
static uint64_t g_lat_max = BT_SHA1_LATENCY_AUTO;
void btsha1_set_latency_batch(uint64_t max_chunks) { __atomic_store_n(&g_lat_max, max_chunks, __ATOMIC_RELAXED); }
uint64_t btsha1_latency_batch_setting() { return __atomic_load_n(&g_lat_max, __ATOMIC_RELAXED); }
uint64_t btsha1_latency_batch() {
  const uint64_t v = btsha1_latency_batch_setting();
  return v == BT_SHA1_LATENCY_AUTO ? (uint64_t)btsha1_device_cus() * 128u : v;
}

// Variant code: NBUF*100 + L*10 + (nt ? 1 : 0).  The product library carries
// ONE hot kernel, the measured default (3-slot ring of one 128-byte line,
// plain loads).  The rejected variants -- other ring shapes,
// non-temporal loads, the LDS-staged kernel -- exist only in the experiments
// library (make experiments: -DBT_SHA1_EXPERIMENTS), where bt_sha1_set_variant
// selects among them; the product's bt_sha1_set_variant accepts only 310.
#ifdef BT_SHA1_EXPERIMENTS
constexpr int kLdsVariant = 1010;  // bt_sha1_set_variant(10, 1, 0): LDS-staged k_sha1_lds
constexpr int kLdsNtVariant = 1011;  // bt_sha1_set_variant(10, 1, 1): the same with nt DMA loads
#define BT_FIXED_VARIANTS(X) X(2, 1, 0) X(3, 1, 0) X(4, 1, 0) X(2, 2, 0) \
  X(2, 1, 2) X(3, 1, 2) X(2, 2, 2)
bool btsha1_experiments_build() { return true; }
#else
#define BT_FIXED_VARIANTS(X) X(3, 1, 0)
bool btsha1_experiments_build() { return false; }
#endif

bool btsha1_fixed_variant_ok(int code) {
#ifdef BT_SHA1_EXPERIMENTS
  if (code == kLdsVariant || code == kLdsNtVariant) return true;
#endif
#define BT_CASE(N, L, A) if (code == N * 100 + L * 10 + (A ? 1 : 0)) return true;
  BT_FIXED_VARIANTS(BT_CASE)
#undef BT_CASE
  return false;
}

hipError_t btsha1_launch_fixed(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                               const uint8_t *d_exp, uint8_t *d_ok, hipStream_t s, int variant, uint32_t tail_len) {
  if (tail_len && d_ok) return hipErrorInvalidValue;  // verify batches are whole chunks
  if (n == 0 && tail_len == 0) return hipSuccess;
  const uint64_t total = n + (tail_len ? 1 : 0);
  // Up to one chunk per CU: a two-wave workgroup per chunk (chain kernel);
  // up to 64 per CU: 64 chunks per two-wave workgroup (latency kernel).
  if (total <= btsha1_chain_batch() && total <= btsha1_latency_batch())
    return btsha1_launch_chain(d_in, nullptr, nullptr, pitch, len, n, d_dig, s, tail_len, d_exp, d_ok);
  if (total <= btsha1_latency_batch()) return launch_lat(d_in, n, pitch, len, d_dig, d_exp, d_ok, s, tail_len);
#ifdef BT_SHA1_EXPERIMENTS
  if (variant == kLdsVariant || variant == kLdsNtVariant) {
    if (n) {
      const hipError_t e = variant == kLdsVariant ? launch_lds<0>(d_in, n, pitch, len, d_dig, d_exp, d_ok, s)
                                                  : launch_lds<2>(d_in, n, pitch, len, d_dig, d_exp, d_ok, s);
      if (e != hipSuccess) return e;
    }
    // The LDS-staged variant has no tail wave: the tail follows on the stream.
    return tail_len ? btsha1_launch_ragged((const uint8_t *)d_in + n * (uint64_t)pitch, nullptr, nullptr, 0, tail_len, 1,
                                           d_dig ? d_dig + 20 * n : nullptr, s)
                    : hipSuccess;
  }
#endif
#define BT_CASE(N, L, A) \
  if (variant == N * 100 + L * 10 + (A ? 1 : 0)) \
    return launch_fixed_v<N, L, A>(d_in, n, pitch, len, d_dig, d_exp, d_ok, s, tail_len);
  BT_FIXED_VARIANTS(BT_CASE)
#undef BT_CASE
  return hipErrorInvalidValue;
}

hipError_t btsha1_launch_fixed_stamped(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                                       uint64_t *d_stamps, hipStream_t s, int variant) {
  if (n == 0) return hipSuccess;
  if (!d_stamps) return hipErrorInvalidValue;
#define BT_CASE(N, L, A) \
  if (variant == N * 100 + L * 10 + (A ? 1 : 0)) \
    return launch_fixed_v<N, L, A>(d_in, n, pitch, len, d_dig, nullptr, nullptr, s, 0u, d_stamps);
  BT_FIXED_VARIANTS(BT_CASE)
#undef BT_CASE
  return hipErrorInvalidValue;  // the LDS variant has no stamped build
}

const char *btsha1_fixed_kernel_name(uint64_t n, int variant) {
  if (n == 0) return "none";
  if (n <= btsha1_chain_batch() && n <= btsha1_latency_batch()) return "k_sha1_chain";
  if (n <= btsha1_latency_batch()) return "k_sha1_lat";
#ifdef BT_SHA1_EXPERIMENTS
  if (variant == kLdsVariant || variant == kLdsNtVariant) return "k_sha1_lds";
#else
  (void)variant;
#endif
  return "k_sha1_fixed";
}

// Ragged batches of at most this many messages take the chain kernel (one
// two-wave workgroup per message; 0: never).  Default: two per CU -- three
// 42 KiB workgroups fit a CU's LDS, and at 2 per CU a lone chain still takes
// 6.07 ms vs 6.71 in k_sha1_lat; at 4 per CU the second round of workgroups
// costs 17.8 ms (tools/latency_bench.py, profiles/r02/latency.txt).
static uint64_t g_chain_max = BT_SHA1_CHAIN_AUTO;
void btsha1_set_chain_batch(uint64_t max_messages) { __atomic_store_n(&g_chain_max, max_messages, __ATOMIC_RELAXED); }
uint64_t btsha1_chain_batch_setting() { return __atomic_load_n(&g_chain_max, __ATOMIC_RELAXED); }
uint64_t btsha1_chain_batch() {
  const uint64_t v = btsha1_chain_batch_setting();
  return v == BT_SHA1_CHAIN_AUTO ? 2ull * btsha1_device_cus() : v;
}

hipError_t btsha1_launch_ragged(const void *d_base, const uint64_t *d_off, const uint32_t *d_len, uint64_t pitch,
                                uint32_t fixed_len, uint64_t n, uint8_t *d_dig, hipStream_t s) {
  if (n == 0) return hipSuccess;
  // A few messages: each one's latency is its serial chain, which the chain
  // kernel runs at ~405 VALU per block instead of the ragged kernel's ~600.
  if (n <= btsha1_chain_batch()) return btsha1_launch_chain(d_base, d_off, d_len, pitch, fixed_len, n, d_dig, s, 0, nullptr, nullptr);
  // Up to 128 messages per CU: the loader / round-wave split of k_sha1_lat.
  if (n <= btsha1_latency_batch()) {
    const uint64_t grid = (n + 63) / 64;
    if (grid > btsha1_device_cus())
      hipLaunchKernelGGL(k_sha1_lat_ragged<3>, dim3((uint32_t)grid), dim3(128), 0, s, (const uint8_t *)d_base, d_off,
                         d_len, pitch, fixed_len, n, d_dig);
    else
      hipLaunchKernelGGL(k_sha1_lat_ragged<2>, dim3((uint32_t)grid), dim3(128), 0, s, (const uint8_t *)d_base, d_off,
                         d_len, pitch, fixed_len, n, d_dig);
    return hipGetLastError();
  }
  // As launch_fixed_v: below one wave per SIMD, one-wave workgroups spread
  // the chains over CUs (each message is a serial chain).
  const uint32_t wg = chain_workgroup(n);
  const uint64_t grid = (n + wg - 1) / wg;
  hipLaunchKernelGGL(k_sha1_ragged, dim3((uint32_t)grid), dim3(wg), 0, s, (const uint8_t *)d_base, d_off,
                     d_len, pitch, fixed_len, n, d_dig);
  return hipGetLastError();
}

hipError_t btsha1_launch_chain_midstate(uint32_t *state, const void *data, uint64_t nblocks, hipStream_t s,
                                        uint32_t *done, uint32_t seq) {
  if (nblocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha1_chain<true>, dim3(1), dim3(128), 0, s, (const uint8_t *)data, nullptr, nullptr, 0ull,
                     nblocks * 64ull, 0ull, state, nullptr, nullptr, nullptr, done, seq);
  return hipGetLastError();
}

hipError_t btsha1_launch_chain_one(const void *msg, uint64_t len, uint8_t *digest, hipStream_t s, uint32_t *done,
                                   uint32_t seq) {
  hipLaunchKernelGGL((k_sha1_chain<false, false>), dim3(1), dim3(128), 0, s, (const uint8_t *)msg, nullptr, nullptr,
                     0ull, len, 0ull, nullptr, digest, nullptr, nullptr, done, seq);
  return hipGetLastError();
}

hipError_t btsha1_launch_chain(const void *base, const uint64_t *offsets, const uint32_t *lens, uint64_t pitch,
                               uint64_t fixed_len, uint64_t n, uint8_t *digests, hipStream_t s, uint64_t tail_len,
                               const uint8_t *expected, uint8_t *ok) {
  const uint64_t grid = n + (tail_len ? 1 : 0);
  if (grid == 0) return hipSuccess;
  if (grid > 0x7fffffffull || (ok && (offsets || tail_len))) return hipErrorInvalidValue;
  if (ok)
    hipLaunchKernelGGL((k_sha1_chain<false, true>), dim3((uint32_t)grid), dim3(128), 0, s, (const uint8_t *)base, offsets,
                       lens, pitch, fixed_len, tail_len, nullptr, digests, expected, ok, nullptr, 0u);
  else
    hipLaunchKernelGGL((k_sha1_chain<false, false>), dim3((uint32_t)grid), dim3(128), 0, s, (const uint8_t *)base,
                       offsets, lens, pitch, fixed_len, tail_len, nullptr, digests, expected, ok, nullptr, 0u);
  return hipGetLastError();
}

hipError_t btsha1_launch_lookup(const uint8_t *d_table, uint64_t n, const uint8_t *d_queries, uint64_t m,
                                uint32_t *d_slots, uint32_t cap, int64_t *d_index, hipStream_t s) {
  hipError_t e = hipMemsetAsync(d_slots, 0, (size_t)cap * 4, s);
  if (e != hipSuccess) return e;
  if (n) hipLaunchKernelGGL(k_lookup_build, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, d_table, n,
                            d_slots, cap - 1);
  if (m) hipLaunchKernelGGL(k_lookup_query, dim3((uint32_t)((m + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, d_table,
                            d_slots, cap - 1, d_queries, m, d_index);
  return hipGetLastError();
}

// Barrier tallies of the -DBT_SHA1_DEBUG_BARRIERS build (g_bar_stats): copy
// them out (and optionally zero them) after a device synchronisation.
// hipErrorNotSupported in the production build, which counts nothing.
hipError_t btsha1_debug_barrier_stats(uint64_t out[3], int reset) {
#ifdef BT_SHA1_DEBUG_BARRIERS
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bar_stats), 3 * sizeof(uint64_t));
  if (e == hipSuccess && reset) {
    const uint64_t zero[3] = {0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_bar_stats), zero, sizeof zero);
  }
  return e;
#else
  (void)out;
  (void)reset;
  return hipErrorNotSupported;
#endif
}

hipError_t btsha1_launch_fill(void *d_buf, uint64_t nbytes, uint64_t first_word, uint64_t seed, hipStream_t s) {
  if (nbytes == 0) return hipSuccess;
  uint64_t pairs = nbytes / 16;
  uint64_t grid = (pairs + kBlock - 1) / kBlock;
  if (grid > 8192) grid = 8192;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(k_fill_synthetic, dim3((uint32_t)grid), dim3(kBlock), 0, s, (uint8_t *)d_buf, nbytes,
                     first_word, seed);
  return hipGetLastError();
}
