#!/usr/bin/env python3
"""Host -> digest rates of the SHA-1 path (BASELINE config 5 / DESIGN.md).

Measures, on one GPU, 512 KiB chunks that start in HOST memory:
  1. bt_sha1_chunks_host on pageable memory (memcpy into pinned staging,
     double-buffered H2D on 2 streams, hot kernel, D2H digests);
  2. the same after bt_sha1_host_register (DMA straight from the image);
  3. raw H2D copy rate of the same bytes (the PCIe ceiling), for reference.
The batched verifier path (util.c:304-337 replacement) is measured by the
verify-stream tool (tools/gpu_session.sh step `stream`).  Prints JSON lines.
"""
import ctypes
import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("btsha1", os.path.join(HERE, "bittorrent-with-congestion-control_amd", "btsha1.py"))
bt = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bt)

CHUNK = 512 * 1024
GIB = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
n = int(GIB * 2**30) // CHUNK
nbytes = n * CHUNK

dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
bt.fill_synthetic(dev.data_ptr(), nbytes, 0, 0x0B175EED)
torch.cuda.synchronize()
host = np.empty(nbytes, dtype=np.uint8)
host[:] = dev.cpu().numpy()
dig_dev = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
bt.chunks_dev(dev.data_ptr(), n, CHUNK, CHUNK, dig_dev.data_ptr())
torch.cuda.synchronize()
want = dig_dev.cpu().numpy().tobytes()
addr = host.ctypes.data


def timed(fn, reps=2):
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, r


t, got = timed(lambda: bt.chunks_host_addr(addr, nbytes))
print(json.dumps({"path": "chunks_host pageable (staging memcpy + 2-stream H2D)", "GiB": GIB,
                  "GiB_per_s": round(GIB / t, 3), "digests_match": got == want}), flush=True)

bt.host_register(addr, nbytes)
t, got = timed(lambda: bt.chunks_host_addr(addr, nbytes))
print(json.dumps({"path": "chunks_host registered (direct DMA, 2-stream H2D overlap)", "GiB": GIB,
                  "GiB_per_s": round(GIB / t, 3), "digests_match": got == want}), flush=True)

pinned_t = torch.from_numpy(host)
torch.cuda.synchronize()
t0 = time.perf_counter()
dev.copy_(pinned_t, non_blocking=True)
torch.cuda.synchronize()
t = time.perf_counter() - t0
print(json.dumps({"path": "raw H2D copy of the registered image (PCIe ceiling)", "GiB": GIB,
                  "GiB_per_s": round(GIB / t, 3)}), flush=True)
bt.host_unregister(addr)
