/*
 * chunk.h -- drop-in replacement header for the reference's chunk.h
 * (yunfanye/Bittorrent-with-Congestion-Control chunk.h:11-39).
 *
 * Same macros and prototypes; callers (make_chunks.c:47, util.c:311,
 * util.c:92,145) compile unchanged against libbtsha1.so.
 */
#ifndef _CHUNK_H_
#define _CHUNK_H_
#include <stdio.h>
#include <inttypes.h>

#define BT_CHUNK_SIZE (512 * 1024)

#define ascii2hex(ascii, len, buf) hex2binary((ascii), (len), (buf))
#define hex2ascii(buf, len, ascii) binary2hex((buf), (len), (ascii))

#ifdef __cplusplus
extern "C" {
#endif
/* chunk.h:25 -- hash fp in BT_CHUNK_SIZE pieces (short last piece), digest i
 * into chunk_hashes[i].  Returns the number of chunks, -1 on error (the
 * reference documents -1 but never returns it; here a GPU error does). */
int make_chunks(FILE *fp, uint8_t **chunk_hashes);

/* chunk.h:28 -- SHA-1 of len bytes into target[20], computed on the GPU by
 * one synchronous chain-kernel call.  Like the reference, which zeroes its
 * context before returning (chunk.c:48), it leaves no copy of the message or
 * of the chaining state behind: the pinned staging the kernel read them from
 * is zeroed before the call returns. */
void shahash(uint8_t *chr, int len, uint8_t *target);

/* chunk.h:31 -- lowercase hex, NUL-terminated (ascii holds 2*len+1). */
void binary2hex(uint8_t *buf, int len, char *ascii);

/* chunk.h:34 -- hex text (len characters) to len/2 bytes, unvalidated. */
void hex2binary(char *hex, int len, uint8_t *buf);
#ifdef __cplusplus
}
#endif

#endif /* _CHUNK_H_ */
