/*
 * verify-stream -- the received-chunk verify path of the peer (util.c:250-337)
 * driven through the batched GPU verifier, end to end from host memory.
 *
 *   verify-stream [-b batch] [-s streams] [-r rounds] [-w warmup-rounds] [-p poll-every]
 *                 [-g verifiers] [-t] [-x] [-z] <data-file> <chunks-file>
 *
 * For every chunk listed in <chunks-file> ("<id> <hex>" lines, as
 * parse_has_get_chunk_file reads them, util.c:90-93) the chunk's bytes are
 * "received" the way save_data_packet assembles them -- 1484-byte DATA
 * payloads memcpy'd into the chunk buffer (util.c:275, common.h:30-31) -- but
 * straight into a pinned verifier slot, then committed with the expected hash
 * (util.c:311-313 becomes a batched GPU verify).  Verdicts are polled from the
 * loop like a select() tick would.  A failed chunk prints "Verification
 * failed!" exactly as util.c:317-318 does.  -x flips one byte of every 7th
 * chunk to exercise the failure branch.  -z ("zero-copy receive") models a
 * receiver that lands DATA payloads directly in the pinned slots (recvfrom
 * into bt_sha1_verifier_slot() + offset): slots are written once, then every
 * later commit re-verifies the bytes already resident in its slot, so the
 * measured rate is the H2D + hash + D2H pipeline alone.  -p N polls for
 * verdicts after every N-th commit (default 1: after each chunk).  -g G runs G
 * verifiers, verifier g on device g % (visible devices), and deals received
 * chunk `id` to verifier id % G; by default one thread drives
 * them all, chunks arriving interleaved across them, and -t gives every
 * verifier a receive thread of its own (the packetized copies of the G
 * verifiers then run side by side).  -w W: the first W rounds are untimed
 * (first touches of the data file's pages, slot pinning); -z with more than
 * one round always leaves round 0 untimed (it lands the data in the slots).
 * The last line is a JSON summary with the host->verdict rate of the timed
 * rounds.
 */
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "bt_sha1.h"
#include "chunk.h"

#define PAYLOAD 1484 /* MAX_PAYLOAD_SIZE, common.h:30 */

/* util.c:316-318 for a failed chunk; tallies verdicts. */
static void count(const bt_sha1_verdict *out, int m, long *good, long *bad) {
  for (int i = 0; i < m; i++) {
    if (out[i].ok) {
      (*good)++;
    } else {
      char h[41];
      binary2hex((uint8_t *)out[i].digest, 20, h);
      printf("Hash: %s\nVerification failed!\n", h);
      (*bad)++;
    }
  }
}

/* -z: which chunk each pinned slot holds (seq = order of the fill in round 0). */
struct resident {
  const uint8_t *slot;
  long seq;
  int k;
};

/* by slot address, then by fill order */
static int cmp_resident(const void *a, const void *b) {
  const struct resident *x = (const struct resident *)a, *y = (const struct resident *)b;
  if (x->slot != y->slot) return x->slot < y->slot ? -1 : 1;
  return x->seq < y->seq ? -1 : x->seq > y->seq;
}

/* by slot address alone (lookups after index_resident) */
static int cmp_slot(const void *a, const void *b) {
  const uint8_t *x = ((const struct resident *)a)->slot, *y = ((const struct resident *)b)->slot;
  return x < y ? -1 : x > y;
}

/* Sort the round-0 fills and keep one entry per slot: the LAST fill of a slot
 * is the chunk resident in it (a poll may recycle a batch inside round 0, so a
 * slot can be handed out twice).  Returns the new count. */
static long index_resident(struct resident *res, long nres) {
  qsort(res, nres, sizeof *res, cmp_resident);
  long m = 0;
  for (long i = 0; i < nres; i++) {
    if (m && res[m - 1].slot == res[i].slot) m--; /* a later fill of the same slot wins */
    res[m++] = res[i];
  }
  return m;
}

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* What every lane reads. */
struct shared {
  const uint8_t *img;
  const int *ids;
  const uint8_t *exp;
  int corrupt, zcopy, poll_every, rounds, warm;
  long ring;
  pthread_barrier_t *bar; /* -t: the lanes meet after the warm-up rounds */
  double *t0;             /* start of the timed rounds */
};

/* One verifier and the chunks routed to it (-g: chunk id modulo G). */
struct lane {
  bt_sha1_verifier *v;
  int *ks;              /* indices into ids[] / exp[] of this verifier's chunks */
  int nk;
  long per_round;       /* commits per round */
  struct resident *res; /* -z: which chunk each of its pinned slots holds */
  long nres;
  long good, bad, total, timed, late_fills, commits;
  int err;
  const struct shared *sh;
};

static int drain_lane(struct lane *l, int wait) {
  bt_sha1_verdict out[256];
  int m;
  while ((m = wait ? bt_sha1_verifier_drain(l->v, out, 256) : bt_sha1_verifier_poll(l->v, out, 256)) > 0)
    count(out, m, &l->good, &l->bad);
  if (m < 0) {
    fprintf(stderr, "verify-stream: %s\n", bt_sha1_last_error());
    return -1;
  }
  return 0;
}

/* The i-th receive of round r on lane l: a slot, the chunk's bytes landed in
 * it (packetized, or only once with -z), the commit, and a poll every
 * poll_every commits. */
static int receive_one(struct lane *l, int r, long i) {
  const struct shared *sh = l->sh;
  int k = l->ks[i % l->nk], fill = 0;
  uint8_t *slot = bt_sha1_verifier_slot(l->v);
  if (!slot) {
    fprintf(stderr, "verify-stream: %s\n", bt_sha1_last_error());
    return -1;
  }
  if (sh->zcopy && r == 0) {
    l->res[l->nres].slot = slot;
    l->res[l->nres].seq = l->nres;
    l->res[l->nres++].k = k;
  } else if (sh->zcopy) {
    struct resident key = {slot, 0, 0}, *hit = bsearch(&key, l->res, l->nres, sizeof *l->res, cmp_slot);
    if (hit) {
      k = hit->k;
    } else if (l->nres < sh->ring) {
      /* A slot round 0 never got: a batch harvested between two slot
       * requests is refilled in place instead of the ring advancing, so
       * which slots round 0 touched depends on timing.  Its first use is its
       * receive: fill it with this commit's chunk and remember it (counted
       * in late_fills: these copies fall inside the timed rounds). */
      long at = 0;
      while (at < l->nres && l->res[at].slot < slot) at++;
      memmove(l->res + at + 1, l->res + at, sizeof *l->res * (size_t)(l->nres - at));
      l->res[at].slot = slot;
      l->res[at].seq = at;
      l->res[at].k = k;
      l->nres++;
      fill = 1;
      if (r >= sh->warm) l->late_fills++;
    } else {
      fprintf(stderr, "verify-stream: more distinct slots than the ring holds (%p)\n", (void *)slot);
      return -1;
    }
  }
  if (!sh->zcopy || r == 0 || fill) {
    const uint64_t off = (uint64_t)sh->ids[k] * BT_CHUNK_SIZE;
    for (uint32_t got = 0; got < BT_CHUNK_SIZE; got += PAYLOAD) { /* save_data_packet, util.c:275 */
      uint32_t len = BT_CHUNK_SIZE - got < PAYLOAD ? BT_CHUNK_SIZE - got : PAYLOAD;
      memcpy(slot + got, sh->img + off + got, len);
    }
    if (sh->corrupt && k % 7 == 3) slot[k % BT_CHUNK_SIZE] ^= 0x5a;
  }
  if (bt_sha1_verifier_commit(l->v, slot, BT_CHUNK_SIZE, sh->exp + 20 * k, (uint64_t)k)) {
    fprintf(stderr, "verify-stream: %s\n", bt_sha1_last_error());
    return -1;
  }
  l->total++;
  if (r >= sh->warm) l->timed++;
  if (++l->commits % sh->poll_every == 0 && drain_lane(l, 0)) return -1;
  return 0;
}

/* End of round r on lane l (before the next round's receives). */
static int round_end(struct lane *l, int r) {
  const struct shared *sh = l->sh;
  if (r + 1 == sh->warm && drain_lane(l, 1)) return -1; /* warm-up done: nothing of it in flight */
  if (sh->zcopy && r == 0) l->nres = index_resident(l->res, l->nres);
  return 0;
}

/* -t: one receive thread per verifier. */
static void *lane_thread(void *arg) {
  struct lane *l = (struct lane *)arg;
  const struct shared *sh = l->sh;
  for (int r = 0; r < sh->rounds; r++) {
    for (long i = 0; i < l->per_round && !l->err; i++)
      if (receive_one(l, r, i)) l->err = 1;
    if (!l->err && round_end(l, r)) l->err = 1;
    if (r + 1 == sh->warm) { /* reached by every lane, failed or not */
      /* every lane has drained its warm-up before the clock starts */
      if (pthread_barrier_wait(sh->bar) == PTHREAD_BARRIER_SERIAL_THREAD) *sh->t0 = now();
      pthread_barrier_wait(sh->bar);
    }
  }
  if (!l->err && drain_lane(l, 1)) l->err = 1;
  return NULL;
}

#define USAGE \
  "usage: %s [-b batch] [-s streams] [-r rounds] [-w warmup-rounds] [-p poll-every] [-g verifiers] [-t] [-x] [-z] " \
  "<data-file> <chunks-file>\n"

int main(int argc, char **argv) {
  int batch = 64, streams = 2, rounds = 1, corrupt = 0, zcopy = 0, poll_every = 1, G = 1, threads = 0, warm = 0, opt;
  while ((opt = getopt(argc, argv, "b:s:r:w:p:g:txz")) != -1) {
    if (opt == 'b') batch = atoi(optarg);
    else if (opt == 's') streams = atoi(optarg);
    else if (opt == 'r') rounds = atoi(optarg);
    else if (opt == 'w') warm = atoi(optarg);
    else if (opt == 'x') corrupt = 1;
    else if (opt == 'z') zcopy = 1;
    else if (opt == 't') threads = 1;
    else if (opt == 'p') poll_every = atoi(optarg) > 0 ? atoi(optarg) : 1;
    else if (opt == 'g') G = atoi(optarg);
    else {
      fprintf(stderr, USAGE, argv[0]);
      return 255;
    }
  }
  if (argc - optind != 2 || G < 1 || G > 64 || rounds < 1 || warm < 0 || batch < 1) {
    fprintf(stderr, USAGE, argv[0]);
    return 255;
  }
  if (zcopy && rounds > 1 && warm < 1) warm = 1; /* round 0 lands the data in the slots */
  if (warm >= rounds) {
    fprintf(stderr, "verify-stream: -w %d leaves no timed round of %d\n", warm, rounds);
    return 255;
  }
  int fd = open(argv[optind], O_RDONLY);
  struct stat st;
  if (fd < 0 || fstat(fd, &st) != 0) {
    perror(argv[optind]);
    return 255;
  }
  const uint8_t *img = st.st_size ? (const uint8_t *)mmap(NULL, st.st_size, PROT_READ, MAP_PRIVATE, fd, 0) : NULL;
  FILE *cf = fopen(argv[optind + 1], "r");
  if (!cf) {
    perror(argv[optind + 1]);
    return 255;
  }
  int cap = 1024, n = 0;
  int *ids = malloc(sizeof(int) * cap);
  uint8_t *exp = malloc(20 * cap);
  char line[256], hex[128];
  while (fgets(line, sizeof line, cf)) {
    int id;
    if (line[0] == '#' || sscanf(line, "%d %127s", &id, hex) != 2 || strlen(hex) != 40) continue;
    if (n == cap) {
      cap *= 2;
      ids = realloc(ids, sizeof(int) * cap);
      exp = realloc(exp, 20 * cap);
    }
    ids[n] = id;
    hex2binary(hex, 40, exp + 20 * n);
    n++;
  }
  fclose(cf);

  /* only whole chunks are verified (util.c:307) */
  int m0 = 0;
  for (int k = 0; k < n; k++)
    if (ids[k] >= 0 && (uint64_t)ids[k] * BT_CHUNK_SIZE + BT_CHUNK_SIZE <= (uint64_t)st.st_size) {
      ids[m0] = ids[k];
      memcpy(exp + 20 * m0, exp + 20 * k, 20);
      m0++;
    }
  n = m0;
  /* -g G: G verifiers, verifier g on device g % (visible devices) -- one per
   * GPU on a node, or G sharing one GPU -- and received chunk `id` goes to
   * verifier id % G (received chunks dealt by index modulo G). */
  const int ndev = bt_sha1_device_count();
  if (ndev <= 0) {
    fprintf(stderr, "verify-stream: no HIP device visible\n");
    return 255;
  }
  double t0 = 0;
  pthread_barrier_t bar;
  struct shared sh = {img, ids, exp, corrupt, zcopy, poll_every, rounds, warm,
                      (long)batch * (streams < 2 ? 2 : streams), &bar, &t0};
  struct lane *L = calloc((size_t)G, sizeof *L);
  long per_round_max = 0;
  for (int g = 0; g < G; g++) {
    L[g].sh = &sh;
    L[g].v = bt_sha1_verifier_create(g % ndev, BT_CHUNK_SIZE, (uint32_t)batch, (uint32_t)streams);
    if (!L[g].v) {
      fprintf(stderr, "verify-stream: %s\n", bt_sha1_last_error());
      return 255;
    }
    L[g].ks = malloc(sizeof(int) * (n ? n : 1));
    for (int k = 0; k < n; k++)
      if (ids[k] % G == g) L[g].ks[L[g].nk++] = k;
    L[g].per_round = L[g].nk;
    if (zcopy) {
      if (L[g].nk == 0 || sh.ring % L[g].nk) {
        fprintf(stderr, "verify-stream -z: batch*streams (%ld) must be a multiple of each verifier's chunk count "
                        "(verifier %d: %d)\n", sh.ring, g, L[g].nk);
        return 255;
      }
      /* which chunk each pinned slot holds.  The verifier hands slots out in
       * ring order, but after a drain it resumes at whichever batch is next,
       * and a batch harvested before the next slot request is refilled in
       * place, so the i-th slot of a later round is not the i-th slot of
       * round 0: every commit is paired with the chunk actually resident in
       * its slot, and a slot first seen after round 0 is filled then. */
      L[g].per_round = sh.ring;
      L[g].res = malloc(sizeof *L[g].res * sh.ring);
    }
    if (L[g].per_round > per_round_max) per_round_max = L[g].per_round;
  }
  int err = 0;
  t0 = now();
  if (threads && G > 1) {
    pthread_barrier_init(&bar, NULL, (unsigned)G);
    pthread_t *th = calloc((size_t)G, sizeof *th);
    for (int g = 0; g < G; g++) pthread_create(&th[g], NULL, lane_thread, &L[g]);
    for (int g = 0; g < G; g++) pthread_join(th[g], NULL);
    free(th);
    pthread_barrier_destroy(&bar);
    for (int g = 0; g < G; g++) err |= L[g].err;
  } else {
    threads = 0;
    /* one receive thread: chunks arrive interleaved across the verifiers, as
     * downloads from several peers would */
    for (int r = 0; r < rounds && !err; r++) {
      for (long i = 0; i < per_round_max && !err; i++)
        for (int g = 0; g < G && !err; g++)
          if (i < L[g].per_round && receive_one(&L[g], r, i)) err = 1;
      for (int g = 0; g < G && !err; g++)
        if (round_end(&L[g], r)) err = 1;
      if (r + 1 == warm) t0 = now();
    }
    for (int g = 0; g < G && !err; g++)
      if (drain_lane(&L[g], 1)) err = 1;
  }
  if (err) return 255;
  double dt = now() - t0;
  long good = 0, bad = 0, total = 0, timed = 0, late = 0;
  for (int g = 0; g < G; g++) {
    good += L[g].good;
    bad += L[g].bad;
    total += L[g].total;
    timed += L[g].timed;
    late += L[g].late_fills;
    bt_sha1_verifier_destroy(L[g].v);
    free(L[g].ks);
    free(L[g].res);
  }
  free(L);
  printf("{\"chunks\": %ld, \"ok\": %ld, \"failed\": %ld, \"seconds\": %.6f, \"GiB_per_s\": %.4f, \"batch\": %d, "
         "\"streams\": %d, \"poll_every\": %d, \"verifiers\": %d, \"devices\": %d, \"receive_threads\": %d, "
         "\"rounds\": %d, \"warmup_rounds\": %d, \"timed_chunks\": %ld, \"late_fills\": %ld, \"mode\": \"%s\"}\n",
         total, good, bad, dt, timed * (double)BT_CHUNK_SIZE / dt / (1u << 30), batch, streams, poll_every, G,
         G < ndev ? G : ndev, threads ? G : 1, rounds, warm, timed, late,
         zcopy ? "zero-copy slots" : "packetized memcpy (util.c:275)");
  return bad && !corrupt ? 1 : 0;
}
