#!/usr/bin/env python3
"""file_bench.py -- end-to-end make-chunks rate from a file (BASELINE config 1's
tool at scale): page-cache-resident file -> host staging ->
H2D -> hot kernel -> "%d %s" lines on stdout.

    python3 tools/file_bench.py [dir] [MiB ...]

For each size (default 1 2048 8192 32768 MiB) writes a file of distinct 512 KiB
chunks under dir (default /dev/shm),
times  make-chunks FILE  (the drop-in make_chunks(FILE*) path: fread into
pinned staging) and  make-chunks -g 0 FILE  (mmap + bt_sha1_chunks_host_multi),
checks the two outputs are identical, and -- where the reference tool built by
oracle/Makefile is present -- times the reference make-chunks on the 1024 MiB
file and checks its output equals ours.  One JSON line per measurement; the
files are removed at the end.  With BT_SHA1_TRACE=1 in the environment the
library prints its per-phase pipeline times to stderr (kept in the log).
"""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MK = os.path.join(HERE, "bittorrent-with-congestion-control_amd", "bin", "make-chunks")
REF_MK = os.path.join(HERE, "oracle", "_ref", "make-chunks")
CHUNK = 512 * 1024


def write_file(path, mib):
    import numpy as np
    rng = np.random.default_rng(0x5EED)
    piece = min(mib, 64)
    block = rng.integers(0, 256, size=piece << 20, dtype=np.uint8)
    with open(path, "wb") as f:
        for i in range(mib // piece):
            for c in range(0, block.size, CHUNK):  # stamp every chunk with its index: chunks differ
                idx = i * (block.size // CHUNK) + c // CHUNK
                block[c:c + 8] = np.frombuffer(idx.to_bytes(8, "little"), dtype=np.uint8)
            f.write(block.tobytes())


def timed(cmd, out_path):
    t0 = time.perf_counter()
    with open(out_path, "wb") as out:
        r = subprocess.run(cmd, stdout=out, stderr=subprocess.PIPE)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        sys.exit(f"{cmd} failed ({r.returncode}): {r.stderr.decode()[-500:]}")
    if r.stderr:
        sys.stderr.write(r.stderr.decode())
    return dt


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "/dev/shm"
    sizes = [int(x) for x in sys.argv[2:]] or [1, 2048, 8192, 32768]
    path = os.path.join(d, f"bt_file_bench_{os.getpid()}.bin")
    outs = [path + s for s in (".gpu", ".gpu_multi", ".ref")]
    try:
        for mib in sizes:
            write_file(path, mib)
            size = os.path.getsize(path)
            timed([MK, path], outs[0])  # page cache + first HIP init out of the way
            for label, cmd, o in (("make-chunks (drop-in make_chunks FILE*)", [MK, path], outs[0]),
                                  ("make-chunks -g 0 (mmap + chunks_host_multi)", [MK, "-g", "0", path], outs[1])):
                dt = timed(cmd, o)
                print(json.dumps({"path": label, "MiB": mib, "seconds": round(dt, 4),
                                  "GiB_per_s": round(size / dt / 2**30, 3),
                                  "note": "process wall time incl. HIP init, file read, H2D, hash, stdout"}), flush=True)
            same = open(outs[0], "rb").read() == open(outs[1], "rb").read()
            print(json.dumps({"MiB": mib, "outputs_identical": same}), flush=True)
            if os.path.exists(REF_MK) and mib == 1024:
                dt = timed([REF_MK, path], outs[2])
                print(json.dumps({"path": "reference make-chunks (CPU, reference Makefile flags)", "MiB": mib,
                                  "seconds": round(dt, 4), "GiB_per_s": round(size / dt / 2**30, 4),
                                  "lines_match_gpu": open(outs[2], "rb").read() == open(outs[0], "rb").read()}),
                      flush=True)
            os.remove(path)
    finally:
        for p in [path] + outs:
            if os.path.exists(p):
                os.remove(p)


if __name__ == "__main__":
    main()
