#!/usr/bin/env python3
"""Checksums of the REFERENCE's digests over whole benchmark batches
(tests/golden/synth_checksums.txt).

Run in the build container only (needs oracle/_ref/libref_sha1.so, compiled
from /root/reference by `make -C oracle`):

    python tests/golden/make_checksums.py [max_chunks]

For the synthetic chunk stream bench.py hashes (chunk g = words
[g*65536, (g+1)*65536) of the frozen generator, seed 0x0B175EED, 512 KiB per
chunk) this hashes chunks 0 .. max_chunks-1 (default 1,048,576 = config 4)
with the reference's own shahash (chunk.c:33-49 over sha.c), on every CPU,
and writes, for each prefix length n the bench and the tests use,

    <n> <SHA-1 of the concatenated 20-byte digests of chunks 0..n-1>

bench.py's `digests_sha1` is that value for its global chunk count (ranks
gather in global order), so its `parity_all_vs_golden` compares EVERY digest
of a run with the reference: 131072 (N=1), 262144 (N=2), 524288 (N=4) and
1,048,576 (N=8, config 4) at the default 131072 chunks per GPU, plus the test
sizes.  The generator is checked against numpy in the CPU tests; the
digests are the reference's.
"""
import ctypes
import hashlib
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_sha1.so")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle_sha1.so")
CHUNK = 512 * 1024
SEED_SYNTH = 0x0B175EED
PREFIXES = [4096, 40960 * 2, 131072, 262144, 40960 * 8, 524288, 1048576]


def main():
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 1048576
    ref = ctypes.CDLL(REF_SO)
    ref.shahash.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    orc = ctypes.CDLL(ORACLE_SO)
    orc.or_fill_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    out = (ctypes.c_uint8 * (20 * total))()
    nth = len(os.sched_getaffinity(0))

    def work(t):
        buf = (ctypes.c_uint8 * CHUNK)()
        for g in range(total * t // nth, total * (t + 1) // nth):
            orc.or_fill_synthetic(buf, CHUNK, g * (CHUNK // 8), SEED_SYNTH)  # ctypes drops the GIL
            ref.shahash(buf, CHUNK, ctypes.byref(out, 20 * g))

    t0 = time.time()
    th = [threading.Thread(target=work, args=(t,)) for t in range(nth)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    raw = bytes(out)
    lines = ["# <n chunks> <sha1 of the concatenated digests of synthetic chunks 0..n-1>, digests by the",
             "# reference's shahash (oracle/_ref/libref_sha1.so); chunk g = splitmix64 words [g*65536, ..),",
             "# seed 0x0B175EED (tests/golden/make_checksums.py)"]
    lines += [f"{n} {hashlib.sha1(raw[:20 * n]).hexdigest()}" for n in PREFIXES if n <= total]
    open(os.path.join(HERE, "synth_checksums.txt"), "w").write("\n".join(lines) + "\n")
    print(f"{total} chunks on {nth} threads in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
