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
round, and how much of the image sits on transparent huge pages
(/proc/self/smaps AnonHugePages of its mapping).  With `torch` as the second
argument the image is instead written the way bench.py writes its host image
(a device-to-host copy into a numpy-backed tensor, 1 GiB at a time).
usage: lock_cost.py [GiB] [torch]
"""
import importlib.util
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
bt = None  # loaded in main(): after torch in `torch` mode, so the library binds to torch's HIP runtime


def load_bt():
    global bt
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


def huge_kib(addr, nbytes):
    """AnonHugePages (KiB) of the mappings overlapping [addr, addr + nbytes)."""
    total, cur = 0, None
    with open("/proc/self/smaps") as f:
        for line in f:
            head = line.split()
            if "-" in head[0] and len(head) >= 5:
                lo, hi = (int(x, 16) for x in head[0].split("-"))
                cur = lo < addr + nbytes and hi > addr
            elif cur and line.startswith("AnonHugePages:"):
                total += int(head[1])
    return total


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    via_torch = len(sys.argv) > 2 and sys.argv[2] == "torch"
    nbytes = int(gib * 2**30)
    src = None
    if via_torch:  # torch's HIP runtime first, as in bench.py (the library then binds to it)
        import torch
        src = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        src.fill_(7)
    load_bt()
    bt.device_count()
    modes = {"one": (nbytes, 1), "seq": (1 << 30, 1), "par": (1 << 30, 8), "par128": (128 << 20, 8)}
    for name, (piece, threads) in modes.items():
        img = np.empty(nbytes, dtype=np.uint8)
        if via_torch:
            import torch
            view = torch.from_numpy(img)
            for o in range(0, nbytes, 1 << 30):
                k = min(1 << 30, nbytes - o)
                view[o:o + k].copy_(src[:k])
        else:
            img[::4096] = 1
        addr = img.ctypes.data
        huge = huge_kib(addr, nbytes)
        first = lock(addr, nbytes, piece, threads)
        again = lock(addr, nbytes, piece, threads)
        print(json.dumps({"mode": name, "written_by": "torch D2H" if via_torch else "numpy", "GiB": gib,
                          "piece_MiB": piece >> 20, "threads": threads, "thp_GiB": round(huge / 2**20, 2),
                          "first_lock_s": first[0], "first_unlock_s": first[1],
                          "again_lock_s": again[0], "again_unlock_s": again[1]}), flush=True)
        del img


if __name__ == "__main__":
    main()
