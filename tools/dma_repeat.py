#!/usr/bin/env python3
"""Run-to-run spread of the direct-DMA host path (registered image) and of a
raw H2D copy of the same image, call after call in one process.

    python3 tools/dma_repeat.py [GiB] [reps]

Prints one JSON line per call: the registered-image bt_sha1_chunks_host rate,
then a raw hipMemcpy of the image into a device buffer kept across calls, and
whether the image's pages sit on the NUMA node of the GPU (numa_maps)."""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "bittorrent-with-congestion-control_amd"))
import btsha1 as bt  # noqa: E402

CHUNK = 512 * 1024
GIB = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n = int(GIB * 2**30) // CHUNK
nbytes = n * CHUNK

dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
bt.fill_synthetic(dev.data_ptr(), nbytes, 0, 0x0B175EED)
torch.cuda.synchronize()
host = np.empty(nbytes, dtype=np.uint8)
host[:] = dev.cpu().numpy()
want = None
addr = host.ctypes.data
bt.host_register(addr, nbytes)
pin = torch.from_numpy(host)
scratch = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
try:
    for r in range(REPS):
        t0 = time.perf_counter()
        got = bt.chunks_host_addr(addr, nbytes)
        dt = time.perf_counter() - t0
        want = want or got
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        scratch.copy_(pin, non_blocking=True)
        torch.cuda.synchronize()
        raw = time.perf_counter() - t1
        print(json.dumps({"rep": r, "registered_GiB_per_s": round(GIB / dt, 3), "raw_h2d_GiB_per_s": round(GIB / raw, 3),
                          "digests_same": got == want}), flush=True)
finally:
    bt.host_unregister(addr)
