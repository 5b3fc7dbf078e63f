/*
 * chunks_ref_harness.c -- TEST ONLY.  Runs the reference's own .chunks
 * parsers and digest lookup (util.c, compiled as it is, with the reference's
 * chunk.c + sha.c) so the tests can compare libbtsha1's replacements with them
 * on the same files:
 *
 *   chunks-ref list   <file>            parse_has_get_chunk_file(file, NULL)  util.c:64-111
 *   chunks-ref master <file>            parse_total_chunk_file(file, NULL)    util.c:113-164
 *   chunks-ref lookup <master> <hexes>  get_chunk_id(hash, table) per query   util.c:28-39
 *
 * list / master print the entry count, then "<id> <40 hex>" per entry
 * (binary2hex, chunk.c:55-61); lookup prints one id (or -1) per query line.
 * Only inputs the reference handles without undefined behaviour are fed to it
 * (no '#' or blank lines: util.c:76-104 counts and fills differently).
 *
 * Built by oracle/Makefile (oracle/_ref/chunks-ref) only where the reference
 * sources exist; util.c's peer/network references are never called and stay
 * unbound (--unresolved-symbols=ignore-in-object-files), as for
 * save_chunk_harness.c.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "util.h"

static void print_table(struct Request *r) {
  char hex[SHA1_HASH_SIZE * 2 + 1];
  printf("%d\n", r->chunk_number);
  for (int i = 0; i < r->chunk_number; i++) {
    binary2hex(r->chunks[i].hash, SHA1_HASH_SIZE, hex);
    printf("%d %s\n", r->chunks[i].id, hex);
  }
}

int main(int argc, char **argv) {
  if (argc >= 3 && !strcmp(argv[1], "list")) {
    struct Request *r = parse_has_get_chunk_file(argv[2], NULL);
    if (!r) return 2;
    print_table(r);
    free_request(r);
    return 0;
  }
  if (argc >= 3 && !strcmp(argv[1], "master")) {
    struct Request *r = parse_total_chunk_file(argv[2], NULL);
    if (!r) return 2;
    print_table(r);
    free_request(r);
    return 0;
  }
  if (argc >= 4 && !strcmp(argv[1], "lookup")) {
    struct Request *r = parse_total_chunk_file(argv[2], NULL);
    FILE *q = fopen(argv[3], "r");
    if (!r || !q) return 2;
    char line[128];
    uint8_t hash[SHA1_HASH_SIZE];
    while (fgets(line, sizeof line, q)) {
      hex2binary(line, SHA1_HASH_SIZE * 2, hash);
      printf("%d\n", get_chunk_id(hash, r));
    }
    fclose(q);
    free_request(r);
    return 0;
  }
  fprintf(stderr, "usage: chunks-ref list|master <file> | lookup <master> <queries>\n");
  return 1;
}
