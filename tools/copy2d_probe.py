#!/usr/bin/env python3
"""tools/copy2d_probe.py -- do strided (2D) host-to-device copies out of a
page-locked image run at the 1D copy's rate?

The host pipeline's last batch could be copied column by column (bytes
[j*W, (j+1)*W) of every chunk, one hipMemcpy2DAsync per column) so that its
chunks' hashing advances while the later columns are still in flight.  That
pays only if a 2D copy with rows of W bytes (source pitch = the chunk length,
destination dense) keeps the DMA engine at its 1D rate.  For a registered
8 GiB image and 1 GiB of it (2048 x 512 KiB chunks): the 1D copy, then the
same bytes as P column copies for P = 2, 4, 8, 16, 32 (rows of 512 KiB / P),
best of 3 each, and the digests of the column-major result checked against
the 1D copy's bytes.
usage: copy2d_probe.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "bittorrent-with-congestion-control_amd"))
import btsha1 as bt  # noqa: E402  (after torch: one HIP runtime)

CHUNK = 512 * 1024
H2D = 1


def main():
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    n = 16384
    img = np.empty(n * CHUNK, dtype=np.uint8)
    img.view(np.uint64)[:] = np.arange(img.size // 8, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    bt.host_register(img.ctypes.data, img.nbytes)
    try:
        L = 2048
        src = img.ctypes.data + (n - L) * CHUNK  # the image's last GiB
        dev = torch.empty(L * CHUNK, dtype=torch.uint8, device="cuda")
        st = torch.cuda.Stream()
        sp = ctypes.c_void_p(st.cuda_stream)

        def timed(fn):
            best = None
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                st.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            return best

        one = timed(lambda: hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(src), L * CHUNK, H2D,
                                               sp))
        print(json.dumps({"copy": "1D", "GiB": 1, "ms": round(one * 1e3, 3),
                          "GiB_per_s": round(1 / one, 2)}), flush=True)
        want = img[(n - L) * CHUNK:].reshape(L, CHUNK)
        for p in (2, 4, 8, 16, 32):
            w = CHUNK // p

            def cols():
                for j in range(p):
                    rc = hip.hipMemcpy2DAsync(ctypes.c_void_p(dev.data_ptr() + j * L * w), w,
                                              ctypes.c_void_p(src + j * w), CHUNK, w, L, H2D, sp)
                    assert rc == 0, rc

            dt = timed(cols)
            got = dev.cpu().numpy().reshape(p, L, w)
            ok = all(np.array_equal(got[j, i], want[i, j * w:(j + 1) * w]) for j in (0, p - 1) for i in (0, L // 2, L - 1))
            print(json.dumps({"copy": "2D columns", "P": p, "row_bytes": w, "rows": L, "ms": round(dt * 1e3, 3),
                              "GiB_per_s": round(1 / dt, 2), "vs_1D": round(one / dt, 3), "bytes_ok": ok}), flush=True)
    finally:
        bt.host_unregister(img.ctypes.data)


if __name__ == "__main__":
    main()
