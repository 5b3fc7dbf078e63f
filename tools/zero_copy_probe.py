#!/usr/bin/env python3
"""tools/zero_copy_probe.py -- how fast do the hash kernels read chunks
straight out of page-locked host memory over PCIe (no DMA copy)?

A host pipeline ends with one chain latency (~6-7 ms) after its last copy:
the last batch's chunks can only be hashed once they have arrived.  Hashing
the final chunks directly from host memory, while the copies of the earlier
ones run, would hide that tail -- if GPU-initiated PCIe reads are fast
enough.  For Z chunks of a registered 8 GiB image:
  * ragged: bt_sha1_ragged_dev with the host image as base (chain kernel up to
    2 x CUs messages, the ragged latency kernel above), kernel time and rate;
  * alone and while a 4 GiB hipMemcpy H2D of other bytes runs beside it.
usage: zero_copy_probe.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "bittorrent-with-congestion-control_amd"))
sys.path.insert(0, os.path.join(HERE, "oracle"))
import btsha1 as bt  # noqa: E402  (after torch: one HIP runtime)
import py_oracle  # noqa: E402  (checker only)

CHUNK = 512 * 1024


def main():
    n = 8192
    img = np.empty(n * CHUNK, dtype=np.uint8)
    img.view(np.uint64)[:] = np.arange(n * CHUNK // 8, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    addr = img.ctypes.data
    bt.host_register(addr, img.nbytes)
    # the device-side address of the registered image (hipHostGetDevicePointer,
    # from the HIP runtime torch loaded -- the one the library binds to)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    dptr = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dptr), ctypes.c_void_p(addr), 0)
    assert rc == 0 and dptr.value, rc
    print(json.dumps({"host_ptr": hex(addr), "device_ptr": hex(dptr.value)}), flush=True)
    base = dptr.value
    dev = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(img[:4 << 30])
    side = torch.cuda.Stream()
    try:
        for z in (64, 256, 512, 1024, 2048):
            first = n - z
            offs = torch.arange(first, n, dtype=torch.int64, device="cuda") * CHUNK
            lens = torch.full((z,), CHUNK, dtype=torch.int32, device="cuda")
            out = torch.zeros(20 * z, dtype=torch.uint8, device="cuda")
            row = {"chunks": z, "kernel": bt.kernel_name(z) if z > 512 else "k_sha1_chain"}
            for beside in (False, True):
                best = None
                for _ in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    if beside:
                        with torch.cuda.stream(side):
                            dev.copy_(src, non_blocking=True)
                    bt.ragged_dev(base, offs.data_ptr(), lens.data_ptr(), z, out.data_ptr())
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                key = "with_4GiB_copy" if beside else "alone"
                row[key + "_ms"] = round(best * 1e3, 3)
                row[key + "_GBps"] = round((z * CHUNK + (4 << 30 if beside else 0)) / best / 1e9, 2)
            got = out.cpu().numpy().tobytes()
            row["digests_ok"] = all(got[20 * i:20 * i + 20] == py_oracle.sha1(img[(first + i) * CHUNK:(first + i + 1) * CHUNK].tobytes())
                                    for i in (0, z // 2, z - 1))
            print(json.dumps(row), flush=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        print(json.dumps({"h2d_4GiB_alone_GBps": round((4 << 30) / (time.perf_counter() - t0) / 1e9, 2)}), flush=True)
    finally:
        bt.host_unregister(addr)


if __name__ == "__main__":
    main()
