// sha1_launch.h -- internal launcher interface between the kernels
// (sha1_kernels.hip) and the C-ABI runtime (bt_sha1_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// n equal chunks of `len` bytes at `pitch` (16-byte multiple, 64*pitch < 4 GiB),
// d_in 16-byte aligned.  d_dig: 20*n bytes (4-byte aligned) or NULL.  When
// d_ok != NULL also compares against d_exp (20*n) and writes one byte per chunk.
// tail_len (0 < tail_len < len, no d_ok): one more chunk of tail_len bytes at
// d_in + n*pitch, digest at d_dig + 20*n, hashed in the same launch.
hipError_t btsha1_launch_fixed(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                               const uint8_t *d_exp, uint8_t *d_ok, hipStream_t s, int variant,
                               uint32_t tail_len = 0);
// Diagnostic build of the hot kernel (variant as above, no verify, no tail):
// lane 0 of every wave writes {s_memtime, s_memrealtime} at the start of its
// loop and after it to d_stamps[4*wave ..] (4 u64 per wave of 64 chunks).
hipError_t btsha1_launch_fixed_stamped(const void *d_in, uint64_t n, uint32_t pitch, uint32_t len, uint8_t *d_dig,
                                       uint64_t *d_stamps, hipStream_t s, int variant);
// Name of the kernel btsha1_launch_fixed runs for a batch of n chunks (tail
// included) on the current device with this variant.
const char *btsha1_fixed_kernel_name(uint64_t n, int variant);
// Batches of at most max_chunks chunks (tail included) take the latency kernel
// k_sha1_lat instead of the selected variant; 0 disables it.  The default,
// BT_SHA1_LATENCY_AUTO, is 128 chunks per CU of the launching device (at
// most two two-wave workgroups per CU; past that the latency kernel loses to
// the hot kernel).
#define BT_SHA1_LATENCY_AUTO UINT64_MAX
void btsha1_set_latency_batch(uint64_t max_chunks);
uint64_t btsha1_latency_batch_setting();  // raw setting (may be BT_SHA1_LATENCY_AUTO)
uint64_t btsha1_latency_batch();          // effective threshold on the current device
#define BT_SHA1_CHAIN_AUTO UINT64_MAX  // = 2 x CUs of the launching device
void btsha1_set_chain_batch(uint64_t max_messages);
uint64_t btsha1_chain_batch_setting();
uint64_t btsha1_chain_batch();
// Compute units of the current device (cached per device; 256 on MI355X).
uint32_t btsha1_device_cus();
// Hot-kernel variant code = ring slots*100 + lines per slot*10 + nt flag.
// The product build knows only 310; the experiments build
// (-DBT_SHA1_EXPERIMENTS) also the rejected ring / nt / LDS-staged variants.
bool btsha1_fixed_variant_ok(int code);
bool btsha1_experiments_build();
// n messages at d_base + d_off[i], d_len[i] bytes each; with d_off == NULL,
// message i is at d_base + i*pitch, fixed_len bytes.  Any alignment.  At most
// btsha1_chain_batch() messages take the chain kernel, more the one-message-
// per-lane ragged kernel.
hipError_t btsha1_launch_ragged(const void *d_base, const uint64_t *d_off, const uint32_t *d_len, uint64_t pitch,
                                uint32_t fixed_len, uint64_t n, uint8_t *d_dig, hipStream_t s);
// Chain kernel (one message per two-wave workgroup; lowest single-chain
// latency).  state / data may be device or pinned host memory.
// done != NULL: after the results, *done = seq is stored with a system-scope
// release, so a host can spin on it instead of waiting on the stream.
hipError_t btsha1_launch_chain_midstate(uint32_t *state, const void *data, uint64_t nblocks, hipStream_t s,
                                        uint32_t *done = nullptr, uint32_t seq = 0);
// One message of len bytes at msg (device or pinned host memory), digest to digest.
hipError_t btsha1_launch_chain_one(const void *msg, uint64_t len, uint8_t *digest, hipStream_t s,
                                   uint32_t *done = nullptr, uint32_t seq = 0);
// n messages: message i at base + (offsets ? offsets[i] : i*pitch), length
// lens ? lens[i] : fixed_len; digest i (big-endian bytes) at digests + 20*i
// (digests may be NULL with ok).  tail_len != 0 (no offsets): one more message
// of tail_len bytes at base + n*pitch.  ok != NULL (no offsets, no tail):
// ok[i] = digest i == expected[20*i ..] (util.c:313).
hipError_t btsha1_launch_chain(const void *base, const uint64_t *offsets, const uint32_t *lens, uint64_t pitch,
                               uint64_t fixed_len, uint64_t n, uint8_t *digests, hipStream_t s, uint64_t tail_len = 0,
                               const uint8_t *expected = nullptr, uint8_t *ok = nullptr);
// One column of n equal chunks (k_sha1_lat's column forms): chunk i's column
// is `width` bytes (a 64-byte multiple) at d_col + i*pitch; d_state holds
// each chunk's chaining state between columns (5 x n words, word k of chunk i
// at d_state[k*n + i], device memory).  FIRST starts from the SHA-1 IV,
// MIDDLE continues, LAST continues and finishes a message of msg_len bytes
// in all (the column ends the message: msg_len is a 64-byte multiple ending
// at it), writing digest i (big-endian, 4-byte aligned) to d_dig + 20*i, and
// with d_ok (LAST only) also ok[i] = digest i == d_exp[20*i ..] (util.c:313;
// d_dig may then be NULL).
#define BTSHA1_COLUMN_FIRST 0
#define BTSHA1_COLUMN_MIDDLE 1
#define BTSHA1_COLUMN_LAST 2
hipError_t btsha1_launch_column(const void *d_col, uint64_t n, uint32_t pitch, uint32_t width, int part,
                                uint32_t *d_state, uint64_t msg_len, uint8_t *d_dig, hipStream_t s,
                                const uint8_t *d_exp = nullptr, uint8_t *d_ok = nullptr);
// Synthetic stream words [first_word, first_word + nbytes/8) into d_buf (16-byte aligned).
hipError_t btsha1_launch_fill(void *d_buf, uint64_t nbytes, uint64_t first_word, uint64_t seed, hipStream_t s);
// Digest lookup: d_index[q] = smallest i with table[i] == queries[q], else -1.
// d_slots: cap (power of two, > n) u32 scratch.
hipError_t btsha1_launch_lookup(const uint8_t *d_table, uint64_t n, const uint8_t *d_queries, uint64_t m,
                                uint32_t *d_slots, uint32_t cap, int64_t *d_index, hipStream_t s);
// Barrier tallies {waves checked, barriers counted, mismatches} of a
// -DBT_SHA1_DEBUG_BARRIERS build (synchronises the device first; reset != 0
// zeroes them); hipErrorNotSupported in the production build.
hipError_t btsha1_debug_barrier_stats(uint64_t out[3], int reset);
