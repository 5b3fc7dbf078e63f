/*
 * sha.h -- drop-in replacement header for the reference's sha.h
 * (yunfanye/Bittorrent-with-Congestion-Control sha.h:29-66).
 *
 * Same context type, constants and prototypes, so callers compile unchanged
 * and link libbtsha1.so instead of sha.o.  SHA1Context keeps the reference's
 * public layout (96 bytes: sha.h:39-50, little-endian default, no
 * RUNTIME_ENDIAN field): hash[] is the chaining state, buffer/bufferLength the
 * byte staging, totalLength the running bit count.  The compression itself
 * runs on the GPU (k_sha1_chain in midstate mode); see bt_sha1.h for the batch API that
 * should be preferred for more than one message.
 */
#ifndef _SHA1_H
#define _SHA1_H

#include <inttypes.h>

#define SHA1_HASH_SIZE 20  /* digest bytes (sha.h:34)                     */
#define SHA1_HASH_WORDS 5  /* digest as big-endian 32-bit words (sha.h:37) */

struct _SHA1Context {
  uint64_t totalLength;             /* message bits absorbed so far      */
  uint32_t hash[SHA1_HASH_WORDS];   /* chaining state                    */
  uint32_t bufferLength;            /* bytes pending in buffer           */
  union {
    uint32_t words[16];
    uint8_t bytes[64];
  } buffer;                         /* partial 64-byte block             */
};

typedef struct _SHA1Context SHA1Context;

#ifdef __cplusplus
extern "C" {
#endif

/* sha.h:58 -- reset to the FIPS 180-1 IV. */
void SHA1Init(SHA1Context *sc);
/* sha.h:59 -- absorb len bytes (whole blocks are compressed on the GPU).
 * The reference burns its stack frame after each call (sha.c:165-174, 526);
 * here the pinned staging the GPU read the blocks and state from is zeroed
 * before SHA1Update / SHA1Final return (the context itself, as in the
 * reference, keeps the partial block until the caller clears it). */
void SHA1Update(SHA1Context *sc, const void *data, uint32_t len);
/* sha.h:60 -- MD-pad, compress the last block(s), write the big-endian digest
 * (hash may be NULL, as in sha.c:545). */
void SHA1Final(SHA1Context *sc, uint8_t hash[SHA1_HASH_SIZE]);

#ifdef __cplusplus
}
#endif

#endif /* _SHA1_H */
