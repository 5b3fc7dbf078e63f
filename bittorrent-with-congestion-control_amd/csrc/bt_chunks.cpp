// bt_chunks.cpp -- the .chunks text formats around the hash path (host code;
// SURVEY.md §8f row 3).  Parsing and formatting only: no hashing here.
//
//   bt_chunks_parse_list    parse_has_get_chunk_file   util.c:64-111
//   bt_chunks_parse_master  parse_total_chunk_file     util.c:113-164
//                           + the "File:" name read of peer.c:299-305
//   bt_chunks_write         make-chunks stdout         make_chunks.c:49-53
//   bt_hex2binary_checked   hex2binary with validation chunk.c:66-83
//
// Deliberate differences from the reference, each of which is a memory-safety
// or silent-garbage bug there:
//   * '#' comment lines are skipped on BOTH passes (the reference skips them
//     when counting, util.c:77-79 / :128-130, but not when filling,
//     util.c:90-104 / :143-157, overrunning its chunk array);
//   * blank lines are skipped (the reference counts them and stores an
//     uninitialised entry);
//   * a hash token must be exactly 40 hex digits (the reference decodes 40
//     characters whatever the token length and accepts non-hex characters);
//     a malformed line is an error reporting its line number.
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bt_sha1.h"
#include "chunk.h"

namespace {

thread_local std::string t_chunks_err;

int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool blank(const char *s) {
  for (; *s; ++s)
    if (!isspace((unsigned char)*s)) return false;
  return true;
}

// "<id> <40 hex>" -> entry; false on a malformed line.
bool parse_line(const char *line, bt_chunk_entry *e) {
  char tok[128];
  int id;
  int used = 0;
  if (sscanf(line, "%d %127s%n", &id, tok, &used) != 2) return false;
  if (!blank(line + used)) return false;
  if (strlen(tok) != 40) return false;
  if (bt_hex2binary_checked(tok, 40, e->hash) != 0) return false;
  e->id = id;
  return true;
}

int64_t parse_body(FILE *f, const char *path, int lineno, bt_chunk_entry **out) {
  std::vector<bt_chunk_entry> v;
  char line[1024];
  while (fgets(line, sizeof line, f)) {
    ++lineno;
    if (line[0] == '#' || blank(line)) continue;
    bt_chunk_entry e;
    if (!parse_line(line, &e)) {
      t_chunks_err = std::string(path) + ":" + std::to_string(lineno) + ": expected \"<id> <40 hex digits>\"";
      return -1;
    }
    v.push_back(e);
  }
  auto *mem = (bt_chunk_entry *)malloc(sizeof(bt_chunk_entry) * (v.empty() ? 1 : v.size()));
  if (!mem) {
    t_chunks_err = "out of memory";
    return -1;
  }
  if (!v.empty()) memcpy(mem, v.data(), sizeof(bt_chunk_entry) * v.size());
  *out = mem;
  return (int64_t)v.size();
}

}  // namespace

extern "C" {

int bt_hex2binary_checked(const char *hex, int len, uint8_t *buf) {
  if (!hex || !buf || len < 0 || (len & 1)) return -1;
  for (int i = 0; i < len; i += 2) {
    const int hi = hexval((unsigned char)hex[i]), lo = hexval((unsigned char)hex[i + 1]);
    if (hi < 0 || lo < 0) return -1;
    buf[i / 2] = (uint8_t)(hi << 4 | lo);
  }
  return 0;
}

int64_t bt_chunks_parse_list(const char *path, bt_chunk_entry **out) {
  if (!path || !out) {
    t_chunks_err = "null pointer";
    return -1;
  }
  FILE *f = fopen(path, "r");
  if (!f) {
    t_chunks_err = std::string("cannot open ") + path;
    return -1;
  }
  const int64_t n = parse_body(f, path, 0, out);
  fclose(f);
  return n;
}

int64_t bt_chunks_parse_master(const char *path, char *data_file, size_t data_file_cap, bt_chunk_entry **out) {
  if (!path || !out) {
    t_chunks_err = "null pointer";
    return -1;
  }
  FILE *f = fopen(path, "r");
  if (!f) {
    t_chunks_err = std::string("cannot open ") + path;
    return -1;
  }
  char l1[1024], l2[1024], name[1024];
  // Two header lines (util.c:125-126): "File: <data file>" (peer.c:299-305) and "Chunks:".
  if (!fgets(l1, sizeof l1, f) || !fgets(l2, sizeof l2, f) || sscanf(l1, "File: %1023s", name) != 1 ||
      strncmp(l2, "Chunks:", 7) != 0) {
    fclose(f);
    t_chunks_err = std::string(path) + ": missing \"File: <name>\" / \"Chunks:\" header";
    return -1;
  }
  if (data_file && data_file_cap) {
    strncpy(data_file, name, data_file_cap - 1);
    data_file[data_file_cap - 1] = 0;
  }
  const int64_t n = parse_body(f, path, 2, out);
  fclose(f);
  return n;
}

void bt_chunks_free(bt_chunk_entry *e) { free(e); }

int bt_chunks_write(void *fp, const char *master_data_file, const uint8_t *digests, int64_t n, int32_t first_id) {
  FILE *f = (FILE *)fp;
  if (!f || (n > 0 && !digests) || n < 0) {
    t_chunks_err = "bad arguments";
    return -1;
  }
  if (master_data_file && fprintf(f, "File: %s\nChunks:\n", master_data_file) < 0) return -1;
  char hex[2 * SHA1_HASH_SIZE + 1];
  for (int64_t i = 0; i < n; ++i) {
    binary2hex((uint8_t *)digests + 20 * i, SHA1_HASH_SIZE, hex);
    if (fprintf(f, "%d %s\n", (int)(first_id + i), hex) < 0) {
      t_chunks_err = "write failed";
      return -1;
    }
  }
  return 0;
}

const char *bt_chunks_last_error(void) { return t_chunks_err.c_str(); }

}  // extern "C"
