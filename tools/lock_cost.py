#!/usr/bin/env python3
"""tools/lock_cost.py -- what page-locking a pageable image costs, first time
and again, and whether it parallelises.

For each mode a FRESH image (np.empty + a write to every page, so the pages
exist but were never locked) is page-locked with bt_sha1_host_register as
  * one:      one call over the whole image;
  * seq:      1 GiB slices one after the other;
  * par:      1 GiB slices, one thread per slice, all at once;
  * par128:   128 MiB slices over 8 threads;
then unlocked, then locked again the same way (`again`: pages locked before).
Each line: seconds to lock, seconds to unlock, and the same for the second
round.  usage: lock_cost.py [GiB]
"""
import importlib.util
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("btsha1", os.path.join(HERE, "bittorrent-with-congestion-control_amd",
                                                                     "btsha1.py"))
bt = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bt)


def lock(addr, nbytes, piece, threads):
    pieces = [(addr + o, min(piece, nbytes - o)) for o in range(0, nbytes, piece)]
    t0 = time.perf_counter()
    if threads <= 1:
        for a, n in pieces:
            bt.host_register(a, n)
    else:
        groups = [pieces[i::threads] for i in range(threads)]
        th = [threading.Thread(target=lambda g=g: [bt.host_register(a, n) for a, n in g]) for g in groups]
        for t in th:
            t.start()
        for t in th:
            t.join()
    t1 = time.perf_counter()
    for a, _ in pieces:
        bt.host_unregister(a)
    return round(t1 - t0, 4), round(time.perf_counter() - t1, 4)


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    nbytes = int(gib * 2**30)
    bt.device_count()
    modes = {"one": (nbytes, 1), "seq": (1 << 30, 1), "par": (1 << 30, 8), "par128": (128 << 20, 8)}
    for name, (piece, threads) in modes.items():
        img = np.empty(nbytes, dtype=np.uint8)
        img[::4096] = 1
        addr = img.ctypes.data
        first = lock(addr, nbytes, piece, threads)
        again = lock(addr, nbytes, piece, threads)
        print(json.dumps({"mode": name, "GiB": gib, "piece_MiB": piece >> 20, "threads": threads,
                          "first_lock_s": first[0], "first_unlock_s": first[1],
                          "again_lock_s": again[0], "again_unlock_s": again[1]}), flush=True)
        del img


if __name__ == "__main__":
    main()
