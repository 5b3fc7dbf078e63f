#!/usr/bin/env python3
"""tools/numa_probe.py -- does the NUMA node of a host image set the rate of
the host paths (config 5)?

The GPU hangs off one socket's PCIe root; a page-locked image whose pages sit
on the other socket's memory is DMA'd across the inter-socket link.  For every
NUMA node: a GiB-sized image first-touched by threads pinned to that node's
CPUs (first touch places the pages), then
  * raw H2D of the registered image (hipMemcpy through torch),
  * bt_sha1_chunks_host on the registered image (direct DMA, 2 streams),
  * bt_sha1_chunks_host on the same image unregistered (staged).
Prints one JSON line per node, with the GPU's own node from sysfs.  With
BT_SHA1_COPY_ORDER=overlap|serial it A/Bs the pipeline's H2D copy order
(profiles/r03/numa_probe.md).
usage: numa_probe.py [GiB]
"""
import importlib.util
import json
import os
import sys
import threading
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("btsha1", os.path.join(HERE, "bittorrent-with-congestion-control_amd",
                                                                     "btsha1.py"))
bt = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bt)
CHUNK = 512 * 1024


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += range(int(a), int(b) + 1)
        elif part:
            out.append(int(part))
    return out


def gpu_node():
    p = torch.cuda.get_device_properties(0)
    bdf = f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}.0"
    try:
        return bdf, int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
    except OSError:
        return bdf, None


def touch_on(arr, cpus, nthreads=8):
    allowed = sorted(set(cpus) & os.sched_getaffinity(0))
    n = arr.nbytes
    step = (n // nthreads + 4095) & ~4095

    def work(i):
        os.sched_setaffinity(0, allowed)  # this thread only
        arr[i * step:min(n, (i + 1) * step)] = 1

    th = [threading.Thread(target=work, args=(i,)) for i in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()


def rate(fn, gib, reps=3):
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return round(gib / best, 3)


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    nbytes = int(gib * 2**30) // CHUNK * CHUNK
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node"))
    bdf, gnode = gpu_node()
    scratch = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for node in nodes:
        cpus = cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read())
        if not set(cpus) & os.sched_getaffinity(0):
            continue
        img = np.empty(nbytes, dtype=np.uint8)
        touch_on(img, cpus)
        addr = img.ctypes.data
        staged = rate(lambda: bt.chunks_host_addr(addr, nbytes), gib)
        bt.host_register(addr, nbytes)
        try:
            direct = rate(lambda: bt.chunks_host_addr(addr, nbytes), gib)
            src = torch.from_numpy(img)

            def h2d():
                scratch.copy_(src, non_blocking=True)
                torch.cuda.synchronize()
            raw = rate(h2d, gib)
        finally:
            bt.host_unregister(addr)
        print(json.dumps({"image_node": node, "gpu": bdf, "gpu_node": gnode, "GiB": round(nbytes / 2**30, 2),
                          "raw_h2d_registered": raw, "chunks_host_registered": direct,
                          "chunks_host_staged": staged}), flush=True)
        del img


if __name__ == "__main__":
    main()
