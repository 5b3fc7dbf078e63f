/*
 * bt_sha1.h -- C-ABI of the MI355X SHA-1 chunk-hashing path (libbtsha1.so).
 *
 * Drop-in surface (declared in sha.h / chunk.h of this directory, which keep
 * the reference's prototypes source-compatible):
 *   SHA1Init / SHA1Update / SHA1Final   replace reference sha.h:58-60
 *   make_chunks / shahash               replace reference chunk.h:25,28
 *   binary2hex / hex2binary             replace reference chunk.h:31,34
 * Every digest is computed by the HIP kernels of
 * bittorrent-with-congestion-control_amd/csrc/ on the GPU; there is no CPU
 * hashing path in this library.  If no GPU / HIP runtime is usable the
 * int-returning entry points return -1 (bt_sha1_last_error() says why) and
 * the void ones (shahash, SHA1Update, SHA1Final) print the error and abort().
 *
 * Additions with no reference counterpart (batching is what makes a GPU pay):
 * device-resident batches, ragged batches, a batched asynchronous verifier
 * that replaces the synchronous shahash + memcmp of util.c:311-313, a host
 * pipeline over pinned buffers, a multi-GPU host split, and the frozen
 * synthetic generator used by the bench and the tests.
 *
 * Conventions: plain pointers and sizes; `stream` is a hipStream_t passed as
 * void* (NULL = the current device's null/default stream, so a call is
 * ordered with the caller's default-stream work, e.g. torch's default stream,
 * exactly like a kernel the caller launches on stream 0); device
 * pointers are prefixed d_, host pointers h_.  Return 0 (or a count) on
 * success, -1 on error.
 */
#ifndef BT_SHA1_H
#define BT_SHA1_H

#include <stddef.h>
#include <stdint.h>

#include "sha.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BT_SHA1_DIGEST_SIZE 20

/* ---- runtime ---------------------------------------------------------- */
/* Number of visible GPUs (0 if none), without creating any context. */
int bt_sha1_device_count(void);
/* Select the device used by the drop-in calls on this thread (default 0). */
int bt_sha1_set_device(int device);
/* Human-readable description of the last error on this thread. */
const char *bt_sha1_last_error(void);
/* Library / kernel build description (arch, ring depth, latency threshold,
 * source id). */
const char *bt_sha1_build_info(void);
/* Id of the kernel sources this library was compiled from (first 16 hex
 * digits of the SHA-256 of sha1_kernels.hip + sha1_device.h, comments
 * stripped, so comment edits keep it): ties profiles
 * (PMC traffic, rocprof summaries) to the build that produced them. */
const char *bt_sha1_source_id(void);
/* Hot-kernel register-ring depth in 128-byte lines (default 3).  The product
 * library carries only the default hot kernel (3 slots of one line, plain
 * loads) and accepts only 3; the measured-and-rejected variants (2 or 4
 * slots, two-line slots, non-temporal loads, and 10 = the LDS-staged
 * k_sha1_lds) are compiled into build_variants/experiments/libbtsha1.so
 * (`make experiments`) alone. */
int bt_sha1_set_ring_depth(int nbuf);
/* Hot-kernel variant: nbuf ring slots of `lines` 128-byte lines each, nt = 1
 * for non-temporal loads.  Returns -1 (message names the experiments
 * library) for a combination this library does not carry: in the product
 * library, anything but (3, 1, 0). */
int bt_sha1_set_variant(int nbuf, int lines, int nt);
/* Batches of at most max_chunks chunks take the latency kernel (a loader /
 * schedule wave and a round wave per 64 chunks, meeting in LDS), which
 * shortens a lone chunk's serial chain; larger batches take the hot-kernel
 * variant above.  0 disables it; UINT64_MAX (the default) = 128 chunks per
 * compute unit of the launching device (32768 on a full MI355X).  Returns the
 * previous setting. */
uint64_t bt_sha1_set_latency_batch(uint64_t max_chunks);
/* Ragged batches (bt_sha1_ragged_dev, strided fallbacks) of at most
 * max_messages messages take the chain kernel -- one two-wave workgroup per
 * message, the lowest latency a single serial chain gets (shahash and the
 * SHA1Update/SHA1Final midstate always use it); larger batches the
 * one-message-per-lane ragged kernel.  0 disables it; UINT64_MAX (default) =
 * two per compute unit.  Returns the previous setting. */
uint64_t bt_sha1_set_chain_batch(uint64_t max_messages);
/* Name of the kernel a fixed-layout batch of n_chunks chunks runs on the
 * current device ("k_sha1_chain" up to two chunks per CU, "k_sha1_lat" up to
 * the latency batch, else "k_sha1_fixed" -- or, in the experiments library
 * with variant 10, "k_sha1_lds");
 * NULL without a device. */
const char *bt_sha1_kernel_name(uint64_t n_chunks);
/* Diagnostic (bench clock measurement): hashes the batch like
 * bt_sha1_chunks_dev through a separately compiled build of the hot kernel
 * whose lane 0 of every wave stores {s_memtime, s_memrealtime} before and
 * after its main loop into d_stamps[4*w .. 4*w+3] (w = chunk index / 64;
 * d_stamps holds 4*ceil(n/64) uint64).  The in-kernel shader clock is
 * delta(memtime) / delta(realtime) * bt_sha1_wallclock_khz().  The production
 * kernel executes no stamp. */
int bt_sha1_clock_probe(const void *d_in, uint64_t n, uint64_t chunk_len, uint64_t pitch, uint8_t *d_digests,
                        uint64_t *d_stamps, void *stream);
/* Rate of s_memrealtime on the current device in kHz (100000 on MI355X). */
int64_t bt_sha1_wallclock_khz(void);
/* Diagnostic (barrier-accounting build, `make dbgbar`): the latency, chain
 * and ragged-latency kernels meet s_barrier from different call sites in
 * their two waves and are correct only while both waves execute the same
 * count.  That build tallies, over every such wave since the last reset,
 * out[0] = waves checked, out[1] = barriers executed, out[2] = waves whose
 * count broke the invariant.  Synchronises the current device first; reset
 * != 0 zeroes the tallies after reading.  Returns -1 in the production
 * library, which counts nothing. */
int bt_sha1_debug_barrier_stats(uint64_t out[3], int reset);

/* Diagnostic: bytes still nonzero in the pinned staging the drop-in calls
 * (shahash, SHA1Update, SHA1Final) copy the message and the chaining state
 * into on `device` -- every call zeroes what it staged before it returns, as
 * the reference leaves no copy behind (chunk.c:48; sha.c:165-174, 526), so
 * this is 0 between calls.  0 when no drop-in call has run on the device;
 * -1 for a negative device.  Scans the whole staging buffer: a test hook, not
 * for hot loops. */
int64_t bt_sha1_debug_dropin_residue(int device);

/* ---- device-resident batches (the hot path) ---------------------------- */
/* n chunks of chunk_len bytes, chunk i at d_in + i*pitch (pitch >= chunk_len).
 * d_digests receives 20*n bytes, digest i = SHA-1(chunk i) as sha.c:545-556
 * serialises it.  Fast path when d_in and pitch are 16-byte aligned and
 * 64*pitch + 4096 <= 4 GiB; any other layout takes the generic kernel. */
int bt_sha1_chunks_dev(const void *d_in, uint64_t n, uint64_t chunk_len, uint64_t pitch,
                       uint8_t *d_digests, void *stream);
/* Same, then compares with d_expected (20*n): d_ok[i] = 1 iff equal
 * (util.c:311-313).  d_digests may be NULL. */
int bt_sha1_verify_dev(const void *d_in, uint64_t n, uint64_t chunk_len, uint64_t pitch,
                       const uint8_t *d_expected, uint8_t *d_ok, uint8_t *d_digests, void *stream);
/* n messages, message i = d_base[d_offsets[i] .. + d_lens[i]). */
int bt_sha1_ragged_dev(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
                       uint64_t n, uint8_t *d_digests, void *stream);
/* Frozen generator: 64-bit word g of the stream = splitmix64(seed + g), LE.
 * Writes words first_word .. into d_buf (16-byte aligned), nbytes bytes. */
int bt_sha1_fill_synthetic(void *d_buf, uint64_t nbytes, uint64_t first_word, uint64_t seed,
                           void *stream);

/* ---- host batches (H2D -> kernel -> D2H, double-buffered pinned staging) - */
/* Page-lock a caller buffer (e.g. an mmap'ed file or a receive ring) so the
 * host batch calls DMA from it directly instead of copying into staging. */
int bt_sha1_host_register(void *h_ptr, uint64_t len);
int bt_sha1_host_unregister(void *h_ptr);
/* make_chunks over a memory image: chunk i = h_in[i*chunk_len ..], the last
 * one may be short.  Returns the chunk count (ceil(total_len/chunk_len)).
 * Memory kept between calls: each device's context keeps its two staging
 * lanes, grown on demand and reused by later calls -- up to 2 x 1 GiB of
 * page-locked host memory (pageable input) and 2 x 1 GiB of HBM.  Pinned or
 * registered input is DMA'd straight from the caller's memory into the same
 * HBM lanes (1 GiB batches).  With BT_SHA1_DMA_BATCH_MB above 1024 the
 * direct-DMA batches are bigger; before the call returns each oversized lane
 * is freed and re-allocated at the size it had before the call (at most the
 * 1 GiB kept lane), so the call leaves exactly the kept lanes allocated.
 * Freeing (hipFree) synchronises the whole device, so such a call returns
 * only after work other streams of this process queued on the GPU has
 * finished. */
int64_t bt_sha1_chunks_host(const void *h_in, uint64_t total_len, uint64_t chunk_len,
                            uint8_t *h_digests);
/* The same split over the first `ndev` GPUs (<=0: all), one host thread per
 * device, contiguous chunk ranges, digests gathered into h_digests in order. */
int64_t bt_sha1_chunks_host_multi(const void *h_in, uint64_t total_len, uint64_t chunk_len,
                                  uint8_t *h_digests, int ndev);
/* The same split over an explicit list of nworkers device ids (SURVEY.md §8e:
 * worker g takes chunks [g*n/G, (g+1)*n/G)).  An id may repeat: each repeat
 * is an independent worker (own host thread, streams and staging) on that
 * device, so the multi-GPU split / staging / ordered gather can be run with
 * any worker count on one GPU.  The first use of a device works in its shared
 * context (kept, as above); the repeats' contexts are freed before the call
 * returns.  At most 64 workers.  Returns the chunk count. */
int64_t bt_sha1_chunks_host_devices(const void *h_in, uint64_t total_len, uint64_t chunk_len,
                                    uint8_t *h_digests, const int *devs, int nworkers);
/* make_chunks over a FILE* with an explicit chunk size (make_chunks uses
 * BT_CHUNK_SIZE).  h_digests must hold 20*ceil(size/chunk_len) bytes. */
int64_t bt_sha1_chunks_file(void *fp /* FILE* */, uint64_t chunk_len, uint8_t *h_digests,
                            uint64_t max_chunks);

/* Where the time of the calling thread's last host pipeline run went
 * (bt_sha1_chunks_host, bt_sha1_chunks_file, make_chunks; for the multi-GPU
 * split, the last worker's run on its own thread), and where its memory sat.
 * The pipeline stages each batch on the host (fill: threaded memcpy / pread
 * into the page-locked staging lanes, or nothing for DMA straight from
 * pinned input), queues its H2D and hash on the lane's stream, and blocks
 * (wait) only when a lane is needed again or at the end.  fill_s close to
 * total_s means the host staging sets the rate; wait_s close to total_s
 * means PCIe / the GPU do.  NUMA fields (Linux sysfs + move_pages): the
 * GPU's node, sampled pages of the staging lanes and of the caller's input
 * per node, and the staging pieces by the node of the CPU their thread ran
 * on; -1 / zeros where unknown.  numa_policy (BT_SHA1_NUMA, applied only
 * when the machine has more than one node and the GPU's node is known):
 * 0 = "off" (pages where the kernel puts them), 1 = "lanes" (the default:
 * the staging lanes and the verifier's receive slots prefer the GPU's
 * node), 2 = "gpu" (that, and the staging threads run on the node's CPUs
 * within the caller's affinity mask -- measured 15-30 % slower on a shared
 * host, where the node's cores are busy with other work: DESIGN.md §6).
 * Pageable input of at least 64 MiB to bt_sha1_chunks_host is page-locked
 * batch by batch (the whole pages of each ~1 GiB batch, all locked before the
 * first copy and released when the call's last batch is done) and DMA'd in
 * place; the unaligned head
 * and tail bytes of each batch, and pages that cannot be locked, are staged
 * (BT_SHA1_PAGEABLE=stage: stage everything).  The last ~batch of chunks of
 * a bt_sha1_chunks_host input (at least 256 MiB of them, chunks of at least
 * 64 KiB; BT_SHA1_COLUMN_MIN_MB) is copied in columns -- 8 strided copies of
 * chunk_len/8 bytes of every chunk (BT_SHA1_COLUMNS: 2..16, 0 = off), for the
 * staged feed gathered into the staging lane by the copy threads -- each
 * hashed into the chunks' chaining state as soon as it has arrived, so the
 * call ends one column's hash, not one whole chunk's, after its last byte
 * crossed PCIe.
 * Returns 0, or -1 when this thread has run no pipeline. */
/* How bt_sha1_chunks_host feeds pageable input of at least 64 MiB to the
 * GPU: page-locked batch by batch and DMA'd in place (REGISTER, the default)
 * or copied into the pinned staging lanes (STAGE; also BT_SHA1_PAGEABLE=stage
 * in the environment).  Process-wide; returns the previous setting or -1. */
#define BT_SHA1_PAGEABLE_REGISTER 0
#define BT_SHA1_PAGEABLE_STAGE 1
int bt_sha1_set_pageable_feed(int feed);
#define BT_SHA1_STATS_NODES 8
typedef struct {
  uint64_t chunks;          /* digests produced                               */
  uint64_t bytes;           /* input bytes                                    */
  uint64_t batch_bytes;     /* bytes per lane batch                           */
  uint32_t batches;         /* lane batches launched                          */
  int32_t staged;           /* 1: copied into the lanes; 0: direct DMA from
                               pinned input; 2: pageable input page-locked
                               batch by batch and DMA'd in place             */
  int32_t device;           /* HIP device                                     */
  int32_t copy_threads;     /* staging threads per piece (BT_SHA1_COPY_THREADS) */
  int32_t numa_nodes;       /* NUMA nodes of the machine (sysfs)              */
  int32_t gpu_numa_node;    /* the GPU's node (-1: unknown)                   */
  int32_t numa_policy;      /* 0 none, 1 lanes, 2 lanes + threads (see above) */
  int32_t registered_batches; /* batches DMA'd from caller pages locked for them */
  uint32_t column_chunks;   /* last chunks copied and hashed column by column
                               (bt_sha1_chunks_host; see above)              */
  double total_s;           /* the whole call                                 */
  double alloc_s;           /* lane allocation / page-locking in the call     */
  double fill_s;            /* providing the input on the host: staging copies
                               / reads, or registering the batch's pages      */
  double wait_s;            /* blocked on a lane's H2D + hash                 */
  double register_s;        /* page-locking caller pages before the first copy
                               (in total_s)                                   */
  double unregister_s;      /* releasing them after the last batch (in total_s) */
  int32_t lane_pages[BT_SHA1_STATS_NODES];  /* sampled staging pages per node */
  int32_t src_pages[BT_SHA1_STATS_NODES];   /* sampled input pages per node   */
  int32_t copy_pieces[BT_SHA1_STATS_NODES]; /* staging pieces per CPU node    */
} bt_sha1_pipeline_stats;
int bt_sha1_get_pipeline_stats(bt_sha1_pipeline_stats *out);

/* ---- batched asynchronous verify (replaces util.c:304-337's hash+memcmp) -- */
typedef struct bt_sha1_verifier bt_sha1_verifier;
typedef struct {
  uint64_t tag;                       /* caller's tag (e.g. chunk id)        */
  int32_t ok;                         /* 1: digest == expected, 0: mismatch  */
  uint8_t digest[BT_SHA1_DIGEST_SIZE]; /* computed digest                    */
} bt_sha1_verdict;

/* batch: chunks per GPU launch; nstreams: batches in flight (>=2 overlaps
 * H2D of batch k+1 with hashing of batch k); chunk_len: BT_CHUNK_SIZE. */
bt_sha1_verifier *bt_sha1_verifier_create(int device, uint32_t chunk_len, uint32_t batch,
                                          uint32_t nstreams);
void bt_sha1_verifier_destroy(bt_sha1_verifier *v);
/* Zero-copy: hand out a pinned chunk_len-byte slot to assemble one chunk in
 * (e.g. save_data_packet's memcpy target, util.c:275).  Several slots may be
 * outstanding (one per in-progress download); blocks only when the ring must
 * wrap onto a batch still in flight.  NULL on error. */
uint8_t *bt_sha1_verifier_slot(bt_sha1_verifier *v);
/* Queue an outstanding slot for verification against expected[20]. */
int bt_sha1_verifier_commit(bt_sha1_verifier *v, uint8_t *slot, uint32_t len,
                            const uint8_t expected[20], uint64_t tag);
/* Give an outstanding slot back unverified (aborted download); no verdict. */
int bt_sha1_verifier_release(bt_sha1_verifier *v, uint8_t *slot);
/* Copying form: slot + memcpy + commit. */
int bt_sha1_verifier_submit(bt_sha1_verifier *v, const void *h_chunk, uint32_t len,
                            const uint8_t expected[20], uint64_t tag);
/* Close the batch being filled; it launches once its outstanding slots are settled. */
int bt_sha1_verifier_flush(bt_sha1_verifier *v);
/* Non-blocking: copy up to max finished verdicts out; returns the count. */
int bt_sha1_verifier_poll(bt_sha1_verifier *v, bt_sha1_verdict *out, int max);
/* Blocking: flush, wait for everything in flight, return up to max verdicts. */
int bt_sha1_verifier_drain(bt_sha1_verifier *v, bt_sha1_verdict *out, int max);
/* Verdicts not yet returned (in flight + finished-unpolled). */
int64_t bt_sha1_verifier_pending(bt_sha1_verifier *v);

/* ---- digest lookup (get_chunk_id / find_chunk, util.c:3-39, on the GPU) - */
/* d_index[q] = smallest i with digest d_table[i] == d_queries[q], else -1.
 * Builds a transient open-addressing table in HBM (stream-ordered alloc). */
int bt_sha1_lookup_dev(const uint8_t *d_table, uint64_t n_table, const uint8_t *d_queries,
                       uint64_t n_queries, int64_t *d_index, void *stream);

/* ---- .chunks files (host-side text formats around the hash) ------------ */
typedef struct {
  int32_t id;                          /* chunk id as written in the file     */
  uint8_t hash[BT_SHA1_DIGEST_SIZE];   /* binary digest                       */
} bt_chunk_entry;

/* "<id> <40 hex>" lines (has/get files; parse_has_get_chunk_file,
 * util.c:64-111).  *out is malloc'ed (bt_chunks_free).  Returns the count or
 * -1 (bt_chunks_last_error()).  '#' and blank lines are skipped; malformed
 * lines are errors (the reference silently stores garbage). */
int64_t bt_chunks_parse_list(const char *path, bt_chunk_entry **out);
/* Master file: "File: <data file>" / "Chunks:" header then list lines
 * (parse_total_chunk_file, util.c:113-164; peer.c:299-305). */
int64_t bt_chunks_parse_master(const char *path, char *data_file, size_t data_file_cap,
                               bt_chunk_entry **out);
void bt_chunks_free(bt_chunk_entry *entries);
/* Write n digests as make-chunks does ("%d %s\n", make_chunks.c:49-53), ids
 * from first_id; with a master header first when master_data_file != NULL. */
int bt_chunks_write(void *fp /* FILE* */, const char *master_data_file, const uint8_t *digests,
                    int64_t n, int32_t first_id);
/* hex2binary (chunk.c:66-83) that rejects non-hex input: 0 or -1. */
int bt_hex2binary_checked(const char *hex, int len, uint8_t *buf);
const char *bt_chunks_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* BT_SHA1_H */
