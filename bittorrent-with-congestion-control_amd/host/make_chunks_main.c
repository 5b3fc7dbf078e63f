/*
 * make-chunks -- .chunks generator over the GPU path (libbtsha1.so).
 *
 * Same command line and stdout as the reference tool (make_chunks.c:14-62):
 *     make-chunks <input-file>      ->  "<id> <40 lowercase hex>\n" per 512 KiB chunk
 * Extra options (no reference counterpart):
 *     -g N   split the file over N GPUs (bt_sha1_chunks_host_multi; 0 = all)
 *     -m     emit a master-chunk-file header first ("File: <path>" / "Chunks:"),
 *            the format parse_total_chunk_file reads (util.c:125-126, peer.c:299-305)
 * Exit status 0 on success, 255 (-1) on any error, as the reference does.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>

#include "bt_sha1.h"
#include "chunk.h"

static void usage(const char *argv0) {
  fprintf(stderr, "usage: %s [-g ngpus] [-m] <input-file>", argv0);
  exit(-1);
}

int main(int argc, char *argv[]) {
  int ngpu = -1, master = 0, opt;
  while ((opt = getopt(argc, argv, "g:m")) != -1) {
    if (opt == 'g') ngpu = atoi(optarg);
    else if (opt == 'm') master = 1;
    else usage(argv[0]);
  }
  if (optind >= argc) usage(argv[0]);
  const char *path = argv[optind];

  struct stat st;
  if (stat(path, &st) != 0) {
    fprintf(stderr, "Can't stat the file %s: %s\n", path, strerror(errno));
    exit(-1);
  }
  /* ceil(size / BT_CHUNK_SIZE) as make_chunks.c:64-76, in integers. */
  const uint64_t size = (uint64_t)st.st_size;
  const uint64_t n = (size + BT_CHUNK_SIZE - 1) / BT_CHUNK_SIZE;
  uint8_t *digests = (uint8_t *)malloc(n ? 20 * n : 20);
  if (!digests) {
    fprintf(stderr, "Out of memory!!!");
    exit(-1);
  }

  int64_t got;
  if (ngpu < 0) {
    /* Single GPU: the reference's own call, make_chunks(FILE*, uint8_t**). */
    FILE *fp = fopen(path, "rb");
    if (!fp) {
      fprintf(stderr, "Can't stat the file %s: %s\n", path, strerror(errno));
      exit(-1);
    }
    uint8_t **rows = (uint8_t **)malloc((n ? n : 1) * sizeof(uint8_t *));
    if (!rows) {
      fprintf(stderr, "Out of memory!!!");
      exit(-1);
    }
    for (uint64_t i = 0; i < n; i++) rows[i] = digests + 20 * i;
    got = make_chunks(fp, rows);
    free(rows);
    fclose(fp);
  } else {
    int fd = open(path, O_RDONLY);
    if (fd < 0) {
      fprintf(stderr, "Can't open the file %s: %s\n", path, strerror(errno));
      exit(-1);
    }
    void *img = size ? mmap(NULL, size, PROT_READ, MAP_PRIVATE, fd, 0) : NULL;
    if (size && img == MAP_FAILED) {
      fprintf(stderr, "Can't map the file %s: %s\n", path, strerror(errno));
      exit(-1);
    }
    got = bt_sha1_chunks_host_multi(img, size, BT_CHUNK_SIZE, digests, ngpu);
    if (size) munmap(img, size);
    close(fd);
  }
  if (got < 0) {
    fprintf(stderr, "make-chunks: %s\n", bt_sha1_last_error());
    exit(-1);
  }

  if (master) printf("File: %s\nChunks:\n", path);
  char ascii[SHA1_HASH_SIZE * 2 + 1];
  for (int64_t i = 0; i < got; i++) {
    hex2ascii(digests + 20 * i, SHA1_HASH_SIZE, ascii);
    printf("%d %s\n", (int)i, ascii);
  }
  free(digests);
  return 0;
}
