#!/usr/bin/env python3
"""file_bench.py -- end-to-end make-chunks rate from a file (BASELINE config 1's
tool at scale): page-cache-resident file -> host staging ->
H2D -> hot kernel -> "%d %s" lines on stdout.

    python3 tools/file_bench.py [GiB] [dir]

Writes a GiB-sized file (distinct 512 KiB chunks) under dir (default /dev/shm),
times  make-chunks FILE  (the drop-in make_chunks(FILE*) path: fread into
pinned staging) and  make-chunks -g 0 FILE  (mmap + bt_sha1_chunks_host_multi),
checks the two outputs are identical, and -- where the reference tool built by
oracle/Makefile is present -- times the reference make-chunks on the first
1 GiB and checks its lines equal ours.  One JSON line per measurement; the file
is removed at the end.
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


def write_file(path, gib):
    import numpy as np
    rng = np.random.default_rng(0x5EED)
    block = rng.integers(0, 256, size=64 << 20, dtype=np.uint8)  # 64 MiB of noise
    with open(path, "wb") as f:
        for i in range(gib * 16):
            block[:8] = np.frombuffer(i.to_bytes(8, "little"), dtype=np.uint8)  # chunks differ
            for c in range(0, block.size, CHUNK):  # stamp every chunk with its index
                block[c:c + 8] = np.frombuffer((i * 128 + c // CHUNK).to_bytes(8, "little"), dtype=np.uint8)
            f.write(block.tobytes())


def timed(cmd, out_path):
    t0 = time.perf_counter()
    with open(out_path, "wb") as out:
        r = subprocess.run(cmd, stdout=out, stderr=subprocess.PIPE)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        sys.exit(f"{cmd} failed ({r.returncode}): {r.stderr.decode()[-500:]}")
    return dt


def main():
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    d = sys.argv[2] if len(sys.argv) > 2 else "/dev/shm"
    path = os.path.join(d, f"bt_file_bench_{os.getpid()}.bin")
    outs = [path + s for s in (".gpu", ".gpu_multi", ".ref", ".small")]
    try:
        write_file(path, gib)
        size = os.path.getsize(path)
        timed([MK, path], outs[0])  # warm the page cache and the GPU context once
        for label, cmd, o in (("make-chunks (drop-in make_chunks FILE*)", [MK, path], outs[0]),
                              ("make-chunks -g 0 (mmap + chunks_host_multi)", [MK, "-g", "0", path], outs[1])):
            dt = timed(cmd, o)
            print(json.dumps({"path": label, "GiB": round(size / 2**30, 3), "seconds": round(dt, 4),
                              "GiB_per_s": round(size / dt / 2**30, 3),
                              "note": "process wall time incl. HIP init, file read, H2D, hash, stdout"}), flush=True)
        same = open(outs[0], "rb").read() == open(outs[1], "rb").read()
        print(json.dumps({"outputs_identical": same}), flush=True)
        if os.path.exists(REF_MK):
            small = path + ".1g"
            with open(path, "rb") as f, open(small, "wb") as g:
                g.write(f.read(1 << 30))
            dt = timed([REF_MK, small], outs[2])
            os.remove(small)
            ref_lines = open(outs[2]).read().splitlines()
            ours = open(outs[0]).read().splitlines()[:len(ref_lines)]
            print(json.dumps({"path": "reference make-chunks (CPU, reference Makefile flags)", "GiB": 1.0,
                              "seconds": round(dt, 4), "GiB_per_s": round(1.0 / dt, 4),
                              "lines_match_gpu": ref_lines == ours}), flush=True)
    finally:
        for p in [path] + outs:
            if os.path.exists(p):
                os.remove(p)


if __name__ == "__main__":
    main()
