/*
 * oracle/sha1_oracle.c -- CPU restatement of the reference SHA-1 chunk path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the "port"
 * CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle_sha1.so.  The product path
 * (libbtsha1.so, HIP) never links or calls anything in here.
 *
 * Pinned against: the reference's own golden vectors (p2-tests/C.chunks:3-6,
 * p2-tests/A.chunks:1-2, p2-tests/B.chunks:1-2, the NIST KATs quoted at
 * sha.c:32-38, the "dash" vector of chunk.c:86-104) and against digests the
 * compiled reference (oracle/_ref, built by oracle/Makefile) produced for
 * edge lengths and synthetic chunks, committed under tests/golden/.
 *
 * What it restates (reference = yunfanye/Bittorrent-with-Congestion-Control,
 * default build: little-endian host, SHA1_UNROLL=20, no SHA1_FAST_COPY):
 *   sha.c:149-163  SHA1Init      -> or_sha1_init
 *   sha.c:176-451  SHA1Guts      -> or_compress   (80-word schedule, 4 round groups)
 *   sha.c:453-527  SHA1Update    -> or_sha1_update (byte-buffered absorb, bit count)
 *   sha.c:529-558  SHA1Final     -> or_sha1_final  (MD padding, BE length, BE digest)
 *   chunk.c:33-49  shahash       -> or_shahash
 *   chunk.c:13-25  make_chunks   -> or_hash_chunks (fixed-size chunks, short tail)
 *   chunk.c:55-83  binary2hex / hex2binary -> or_binary2hex / or_hex2binary
 * plus the frozen synthetic-data generator shared with the device kernel
 * (bt_sha1.h: bt_sha1_fill_synthetic), a pthread batch driver for the CPU
 * baseline, and or_synth_digests: the digests of a whole range of synthetic
 * chunks, each regenerated per thread (no image in memory), so the GPU tests
 * can check every digest of a 64 GiB (config 3) or multi-rank (config 4)
 * batch, not a sample.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t bits;      /* total message length in bits (sha.c:511)      */
  uint32_t h[5];      /* chaining state (sha.h:41)                     */
  uint32_t fill;      /* bytes buffered in blk (sha.h:42)              */
  uint8_t blk[64];    /* partial block (sha.h:43-46)                   */
} or_ctx;

static inline uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* Big-endian word load: sha.c loads host-LE words then BYTESWAPs them
 * (sha.c:186-189); reading the bytes MSB-first is the same value. */
static inline uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

/* One compression, sha.c:176-451.  W[80] expanded up front exactly like the
 * reference's buf[80] (sha.c:191-200); round functions sha.c:52-55, K
 * constants sha.c:66-69. */
static void or_compress(uint32_t h[5], const uint8_t *block) {
  uint32_t w[80];
  for (int t = 0; t < 16; t++) w[t] = be32(block + 4 * t);
  /* The loops stay loops; the unroll hints only let gcc resolve the round
   * selection at compile time (+40 % for the bulk sweeps of or_synth_digests). */
  _Pragma("GCC unroll 64") for (int t = 16; t < 80; t++) w[t] = rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);

  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
  _Pragma("GCC unroll 80") for (int t = 0; t < 80; t++) {
    uint32_t f, k;
    if (t < 20) {
      f = d ^ (b & (c ^ d));
      k = 0x5a827999u;
    } else if (t < 40) {
      f = b ^ c ^ d;
      k = 0x6ed9eba1u;
    } else if (t < 60) {
      f = (b & (c | d)) | (c & d);
      k = 0x8f1bbcdcu;
    } else {
      f = b ^ c ^ d;
      k = 0xca62c1d6u;
    }
    uint32_t tmp = rol(a, 5) + f + e + w[t] + k;
    e = d;
    d = c;
    c = rol(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
}

void or_sha1_init(or_ctx *c) {
  c->bits = 0;
  c->h[0] = 0x67452301u;
  c->h[1] = 0xefcdab89u;
  c->h[2] = 0x98badcfeu;
  c->h[3] = 0x10325476u;
  c->h[4] = 0xc3d2e1f0u;
  c->fill = 0;
}

/* Byte-buffered absorb (sha.c:502-522): every byte goes through the 64-byte
 * staging block, the bit counter advances by 8 per byte. */
void or_sha1_update(or_ctx *c, const void *data, uint32_t len) {
  const uint8_t *p = (const uint8_t *)data;
  while (len) {
    uint32_t take = 64u - c->fill;
    if (take > len) take = len;
    memcpy(c->blk + c->fill, p, take);
    c->bits += (uint64_t)take * 8u;
    c->fill += take;
    p += take;
    len -= take;
    if (c->fill == 64u) {
      or_compress(c->h, c->blk);
      c->fill = 0;
    }
  }
}

/* MD padding + digest serialisation (sha.c:529-558). */
void or_sha1_final(or_ctx *c, uint8_t out[20]) {
  static const uint8_t pad0[64] = {0x80};
  uint32_t npad = 120u - c->fill;
  if (npad > 64u) npad -= 64u;
  uint64_t bits = c->bits;
  uint8_t lenbe[8];
  for (int i = 0; i < 8; i++) lenbe[i] = (uint8_t)(bits >> (56 - 8 * i));
  or_sha1_update(c, pad0, npad);
  or_sha1_update(c, lenbe, 8);
  for (int i = 0; i < 5; i++) {
    out[4 * i + 0] = (uint8_t)(c->h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(c->h[i] >> 8);
    out[4 * i + 3] = (uint8_t)(c->h[i]);
  }
}

/* chunk.c:33-49 (int length, as the reference takes it). */
void or_shahash(const uint8_t *buf, int len, uint8_t out[20]) {
  or_ctx c;
  or_sha1_init(&c);
  or_sha1_update(&c, buf, (uint32_t)len);
  or_sha1_final(&c, out);
  memset(&c, 0, sizeof c);
}

/* Midstate form used by the tests of the streaming API: compress nblocks full
 * blocks into h (no padding). */
void or_sha1_blocks(uint32_t h[5], const uint8_t *blocks, uint64_t nblocks) {
  for (uint64_t i = 0; i < nblocks; i++) or_compress(h, blocks + 64 * i);
}

/* chunk.c:55-61: lowercase "%.2x" per byte, NUL-terminated. */
void or_binary2hex(const uint8_t *buf, int len, char *hex) {
  static const char dig[] = "0123456789abcdef";
  for (int i = 0; i < len; i++) {
    hex[2 * i] = dig[buf[i] >> 4];
    hex[2 * i + 1] = dig[buf[i] & 15];
  }
  hex[2 * len] = 0;
}

/* chunk.c:66-83: toupper, then '0'..'9' or 'A'-10; no validation. */
static uint8_t nib(char ch) {
  if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 'a' + 'A');
  return (uint8_t)((ch <= '9') ? (ch - '0') : (ch - ('A' - 10)));
}
void or_hex2binary(const char *hex, int len, uint8_t *buf) {
  for (int i = 0; i < len; i += 2) buf[i / 2] = (uint8_t)((nib(hex[i]) << 4) | nib(hex[i + 1]));
}

/* ---- frozen synthetic generator (mirrors bt_sha1_fill_synthetic) -----------
 * 64-bit word g of the global stream = splitmix64(seed + g), little-endian.
 * Chunk i of length L occupies words [i*L/8, (i+1)*L/8) of the stream, so a
 * 512 KiB chunk i is words i*65536 .. i*65536+65535. */
static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
void or_fill_synthetic(uint8_t *buf, uint64_t nbytes, uint64_t first_word, uint64_t seed) {
  uint64_t nw = nbytes / 8;
  for (uint64_t i = 0; i < nw; i++) {
    uint64_t v = splitmix64(seed + first_word + i);
    memcpy(buf + 8 * i, &v, 8); /* host is little-endian */
  }
  uint64_t rem = nbytes - 8 * nw;
  if (rem) {
    uint64_t v = splitmix64(seed + first_word + nw);
    memcpy(buf + 8 * nw, &v, rem);
  }
}

/* ---- batch driver (CPU baseline + bulk parity) ----------------------------
 * Hash n chunks of chunk_len bytes laid out at a fixed pitch, the last chunk
 * possibly shorter (last_len), like make_chunks' fread loop (chunk.c:20-22).
 * nthreads > 1 splits the chunk index range statically across pthreads. */
typedef struct {
  const uint8_t *base;
  uint64_t pitch;
  uint64_t lo, hi, n;
  uint32_t chunk_len, last_len;
  uint8_t *out;
} or_job;

static void *or_worker(void *arg) {
  or_job *j = (or_job *)arg;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    uint32_t len = (i + 1 == j->n) ? j->last_len : j->chunk_len;
    or_shahash(j->base + i * j->pitch, (int)len, j->out + 20 * i);
  }
  return NULL;
}

/* Run worker(jobs[t]) for t < nthreads: job 0 on the calling thread, the
 * others on pthreads.  A thread that fails to start is never joined (its
 * pthread_t is unset); the call then returns -1 after joining the threads
 * that did start, so the caller reports a clean failure instead of reading a
 * partly written output. */
static int or_run_jobs(void *(*worker)(void *), void *jobs, size_t job_size, int nthreads) {
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  unsigned char *started = (unsigned char *)calloc((size_t)nthreads, 1);
  if (!th || !started) {
    free(th);
    free(started);
    return -1;
  }
  int failed = 0;
  for (int t = 1; t < nthreads; t++) {
    if (pthread_create(&th[t], NULL, worker, (char *)jobs + (size_t)t * job_size) == 0)
      started[t] = 1;
    else
      failed = 1;
  }
  worker(jobs);
  for (int t = 1; t < nthreads; t++)
    if (started[t]) pthread_join(th[t], NULL);
  free(th);
  free(started);
  return failed ? -1 : 0;
}

int or_hash_chunks(const uint8_t *base, uint64_t n, uint64_t pitch, uint32_t chunk_len,
                   uint32_t last_len, uint8_t *out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  or_job *jobs = (or_job *)calloc((size_t)nthreads, sizeof(or_job));
  if (!jobs) return -1;
  for (int t = 0; t < nthreads; t++)
    jobs[t] = (or_job){base, pitch, n * t / nthreads, n * (t + 1) / nthreads, n, chunk_len, last_len, out};
  const int rc = or_run_jobs(or_worker, jobs, sizeof(or_job), nthreads);
  free(jobs);
  return rc;
}

/* ---- digests of synthetic chunks, regenerated on the fly ---------------------
 * Chunk g (global index) of chunk_len bytes = stream words [g*chunk_len/8, ..)
 * (chunk_len a multiple of 8, as bench.py lays chunks out at pitch = length).
 * out[20*i ..] = shahash of chunk first_chunk + i, i < n; nthreads pthreads,
 * each regenerating its chunks into its own chunk_len-byte scratch buffer. */
typedef struct {
  uint64_t first, lo, hi, seed;
  uint32_t chunk_len;
  uint8_t *out;
  int err;
} or_synth_job;

static void *or_synth_worker(void *arg) {
  or_synth_job *j = (or_synth_job *)arg;
  uint8_t *buf = (uint8_t *)malloc(j->chunk_len ? j->chunk_len : 1);
  if (!buf) {
    j->err = 1;
    return NULL;
  }
  for (uint64_t i = j->lo; i < j->hi; i++) {
    or_fill_synthetic(buf, j->chunk_len, (j->first + i) * (j->chunk_len / 8), j->seed);
    or_shahash(buf, (int)j->chunk_len, j->out + 20 * i);
  }
  free(buf);
  return NULL;
}

int or_synth_digests(uint64_t first_chunk, uint64_t n, uint32_t chunk_len, uint64_t seed, uint8_t *out,
                     int nthreads) {
  if (chunk_len % 8) return -1;
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  or_synth_job *jobs = (or_synth_job *)calloc((size_t)nthreads, sizeof(or_synth_job));
  if (!jobs) return -1;
  for (int t = 0; t < nthreads; t++)
    jobs[t] = (or_synth_job){first_chunk, n * t / nthreads, n * (t + 1) / nthreads, seed, chunk_len, out, 0};
  int err = or_run_jobs(or_synth_worker, jobs, sizeof(or_synth_job), nthreads);
  for (int t = 0; t < nthreads; t++) err |= jobs[t].err;  /* jobs that never started keep err = 0 */
  free(jobs);
  return err ? -1 : 0;
}
