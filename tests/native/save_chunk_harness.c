/*
 * save_chunk_harness.c -- drives the reference peer's UNMODIFIED receive /
 * verify code (util.c, the hash's caller #2) linked against libbtsha1.so
 * instead of the reference's chunk.o + sha.o (reference Makefile:6).
 *
 * Built by `make dropin` (only where the reference sources exist) as
 * oracle/_ref/save-chunk-dropin from $(REF)/util.c + $(REF)/file.c, compiled
 * as they are, plus this file.  No socket, no peer loop: the harness plays
 * the part of peer.c's event loop for one GET:
 *   start-up      has_chunk_table  = parse_has_get_chunk_file(has, NULL)   (peer.c:289)
 *                 total_chunk_table = parse_total_chunk_file(master, NULL)
 *   GET           create_file(out, BT_CHUNK_SIZE); current_request =
 *                 parse_has_get_chunk_file(get, out)                        (peer.c:246-249, 228)
 *   per DATA      save_data_packet(packet, chunk)                           (util.c:250-277)
 *   chunk done    save_chunk(chunk) -> shahash (util.c:311) -> memcmp (:313)
 * Deliveries: every chunk of the GET in order, with the chunk given by -c
 * delivered first with one byte flipped (must fail verification and return
 * to NOT_STARTED, util.c:316-319) and then again intact.  After each
 * save_chunk the harness prints "STATE <index> <state>".
 *
 *   save-chunk-dropin [-c corrupt_index] <data-file> <master.chunks> <get.chunks> <has.chunks> <out-file>
 *
 * util.c's crash-recovery functions reference peer/network symbols
 * (send_packet, start_download, ...) that are never called here; the link
 * leaves them unbound (--unresolved-symbols=ignore-in-object-files) rather
 * than linking the reference's network code.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "util.h"

static int deliver(const unsigned char *img, int index, int corrupt) {
  struct Chunk *c = &current_request->chunks[index];
  const long base = (long)c->id * BT_CHUNK_SIZE;
  unsigned char pkt[MAX_PACKET_SIZE];
  c->state = RECEIVING; /* as pick_a_chunk / the GET handshake leaves it */
  unsigned int seq = 1;
  for (int off = 0; off < BT_CHUNK_SIZE; off += MAX_PAYLOAD_SIZE, ++seq) {
    const int len = BT_CHUNK_SIZE - off < MAX_PAYLOAD_SIZE ? BT_CHUNK_SIZE - off : MAX_PAYLOAD_SIZE;
    memset(pkt, 0, HEADER_LENGTH);
    *(unsigned short *)(pkt + 0) = htons(MAGIC_NUMBER);
    pkt[2] = VERSION_NUMBER;
    pkt[3] = DATA;
    *(unsigned short *)(pkt + 4) = htons(HEADER_LENGTH);
    *(unsigned short *)(pkt + 6) = htons((unsigned short)(HEADER_LENGTH + len));
    *(unsigned int *)(pkt + 8) = htonl(seq);
    memcpy(pkt + HEADER_LENGTH, img + base + off, len);
    if (corrupt && off == 0) pkt[HEADER_LENGTH + 7] ^= 0x5a;
    save_data_packet((struct packet *)pkt, index);
  }
  const int r = save_chunk(index);
  printf("STATE %d %d\n", index, c->state);
  fflush(stdout);
  return r;
}

int main(int argc, char **argv) {
  int corrupt = -1, opt;
  while ((opt = getopt(argc, argv, "c:")) != -1) {
    if (opt == 'c') corrupt = atoi(optarg);
    else return 255;
  }
  if (argc - optind != 5) {
    fprintf(stderr, "usage: %s [-c idx] <data-file> <master.chunks> <get.chunks> <has.chunks> <out-file>\n", argv[0]);
    return 255;
  }
  char *data = argv[optind], *master = argv[optind + 1], *get = argv[optind + 2], *has = argv[optind + 3];
  char out[FILE_NAME_SIZE];
  memset(out, 0, sizeof out);
  strncpy(out, argv[optind + 4], sizeof out - 1);

  FILE *f = fopen(data, "rb");
  if (!f) return 255;
  fseek(f, 0, SEEK_END);
  const long size = ftell(f);
  fseek(f, 0, SEEK_SET);
  unsigned char *img = malloc(size > 0 ? size : 1);
  if (fread(img, 1, size, f) != (size_t)size) return 255;
  fclose(f);

  has_chunk_table = parse_has_get_chunk_file(has, NULL);
  total_chunk_table = parse_total_chunk_file(master, NULL);
  create_file(out, BT_CHUNK_SIZE);
  current_request = parse_has_get_chunk_file(get, out);
  if (!has_chunk_table || !total_chunk_table || !current_request) {
    fprintf(stderr, "cannot parse chunk files\n");
    return 255;
  }
  for (int i = 0; i < current_request->chunk_number; ++i) {
    if ((long)(current_request->chunks[i].id + 1) * BT_CHUNK_SIZE > size) return 255;
    if (i == corrupt) deliver(img, i, 1);
    deliver(img, i, 0);
  }
  printf("ALL_FINISHED %d\n", all_chunk_finished());
  free(img);
  return 0;
}
