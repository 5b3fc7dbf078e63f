#!/usr/bin/env python3
"""Generate the committed golden vectors under tests/golden/ from the REFERENCE.

Run in the build container only (needs /root/reference and the reference
objects that `make -C oracle` compiles from it into oracle/_ref/):

    make -C oracle && python tests/golden/make_golden.py

Every expected digest written here comes from the reference's own code:
  * oracle/_ref/libref_sha1.so  = reference chunk.c + sha.c (shahash, SHA1*)
  * oracle/_ref/make-chunks     = reference make_chunks.c + chunk.c + sha.c
Inputs are either the reference's own data files (C.tar and the .chunks
fixtures of p2-tests/, copied as data) or the frozen synthetic generator
(oracle/sha1_oracle.c: or_fill_synthetic == bt_sha1_fill_synthetic), which is
pure integer arithmetic and is itself checked against numpy in the CPU tests.
"""
import ctypes
import hashlib
import lzma
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("BT_REFERENCE", "/root/reference")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_sha1.so")
REF_MK = os.path.join(REPO, "oracle", "_ref", "make-chunks")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle_sha1.so")

CHUNK = 512 * 1024
SEED_SYNTH = 0x0B175EED  # config 2
SEED_EDGE = 0x5EED0001
SEED_TAIL = 0x7A11
SEED_RAGGED = 0xABCD
EDGE_LENGTHS = [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 121, 127, 128, 129, 1000,
                4095, 4096, 65536, 524287, 524288, 524289, 1048576 + 12345]
N_RAGGED = 96


def ragged_len(k):
    return (k * 7919) % 2113 + (k % 5) * 64


def load():
    ref = ctypes.CDLL(REF_SO)
    ref.shahash.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    ref.SHA1Init.argtypes = [ctypes.c_void_p]
    ref.SHA1Update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    ref.SHA1Final.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    orc = ctypes.CDLL(ORACLE_SO)
    orc.or_fill_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    return ref, orc


def ref_hash(ref, data: bytes) -> str:
    buf = ctypes.create_string_buffer(data, len(data) + 1)
    out = ctypes.create_string_buffer(20)
    ref.shahash(buf, len(data), out)
    return out.raw.hex()


def synth(orc, nbytes, first_word, seed) -> bytes:
    buf = ctypes.create_string_buffer(max(nbytes, 1))
    orc.or_fill_synthetic(buf, nbytes, first_word, seed)
    return buf.raw[:nbytes]


def main():
    if not os.path.exists(os.path.join(REF, "sha.c")):
        sys.exit("reference not present; golden vectors are generated in the build container only")
    ref, orc = load()

    # -- KATs: NIST (sha.c:32-38 via its SHA1_TEST main), "dash" (chunk.c:86-104), extra patterns
    kat = []
    ctx = ctypes.create_string_buffer(128)
    out = ctypes.create_string_buffer(20)
    ref.SHA1Init(ctx)
    block = b"a" * 1000
    for _ in range(1000):
        ref.SHA1Update(ctx, block, 1000)
    ref.SHA1Final(ctx, out)
    kat.append(("million_a", 1000000, out.raw.hex()))
    for name, data in [("abc", b"abc"),
                       ("nist448", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"),
                       ("dash", b"dash"), ("empty", b""),
                       ("zeros_512k", bytes(CHUNK)), ("ff_512k", b"\xff" * CHUNK),
                       ("iota_512k", bytes(i & 255 for i in range(CHUNK)))]:
        kat.append((name, len(data), ref_hash(ref, data)))
    with open(os.path.join(HERE, "kat.txt"), "w") as f:
        f.write("# name length sha1  (expected = reference sha.c via shahash/SHA1*)\n")
        for name, n, h in kat:
            assert h == hashlib.sha1(b"a" * n if name == "million_a" else
                                     {"abc": b"abc", "dash": b"dash", "empty": b"",
                                      "nist448": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
                                      "zeros_512k": bytes(CHUNK), "ff_512k": b"\xff" * CHUNK,
                                      "iota_512k": bytes(i & 255 for i in range(CHUNK))}[name]).hexdigest()
            f.write(f"{name} {n} {h}\n")

    # -- edge lengths over the synthetic stream (seed SEED_EDGE, word 0)
    stream = synth(orc, max(EDGE_LENGTHS), 0, SEED_EDGE)
    with open(os.path.join(HERE, "edge_lengths.txt"), "w") as f:
        f.write(f"# length sha1 of synthetic stream prefix (seed {SEED_EDGE:#x}, first_word 0)\n")
        for n in EDGE_LENGTHS:
            f.write(f"{n} {ref_hash(ref, stream[:n])}\n")

    # -- ragged batch: message k = synthetic(seed SEED_RAGGED, first_word k*1024), length ragged_len(k)
    with open(os.path.join(HERE, "ragged.txt"), "w") as f:
        f.write(f"# k length sha1 ; message k = synthetic(seed {SEED_RAGGED:#x}, first_word k*1024)[:length]\n")
        for k in range(N_RAGGED):
            n = ragged_len(k)
            f.write(f"{k} {n} {ref_hash(ref, synth(orc, n, k * 1024, SEED_RAGGED))}\n")

    # -- config 2: 4096 synthetic 512 KiB chunks, chunk i = words i*65536.. (seed SEED_SYNTH)
    n = 4096
    per = 256
    with open(os.path.join(HERE, "synth4096.txt"), "w") as f:
        f.write(f"# chunk sha1 ; chunk i = synthetic(seed {SEED_SYNTH:#x}, first_word i*65536)[:524288]\n")
        for base in range(0, n, per):
            data = synth(orc, per * CHUNK, base * (CHUNK // 8), SEED_SYNTH)
            for i in range(per):
                f.write(f"{base + i} {ref_hash(ref, data[i * CHUNK:(i + 1) * CHUNK])}\n")

    # -- make-chunks stdout (config 1 plumbing): C.tar and a short-tail synthetic file
    with tempfile.TemporaryDirectory() as td:
        tail = os.path.join(td, "tail.bin")
        with open(tail, "wb") as g:
            g.write(synth(orc, 3 * CHUNK + 12345, 0, SEED_TAIL))
        for src, dst in [(os.path.join(REF, "C.tar"), "C.tar.make-chunks.out"),
                         (os.path.join(REF, "p2-tests", "A.tar"), "A.tar.make-chunks.out"),
                         (tail, "tail.make-chunks.out")]:
            res = subprocess.run([REF_MK, src], check=True, capture_output=True)
            with open(os.path.join(HERE, dst), "wb") as g:
                g.write(res.stdout)

    # -- the reference's own fixture data files (data, copied verbatim)
    for rel in ["p2-tests/C.chunks", "p2-tests/A.chunks", "p2-tests/B.chunks", "p2-tests/test1.chunks"]:
        shutil.copyfile(os.path.join(REF, rel), os.path.join(HERE, "ref_" + os.path.basename(rel)))
    with open(os.path.join(REF, "C.tar"), "rb") as g:
        ctar = g.read()
    with open(os.path.join(HERE, "C.tar.xz"), "wb") as g:
        g.write(lzma.compress(ctar, preset=9))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
