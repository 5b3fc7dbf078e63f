#!/usr/bin/env python3
"""tools/numa_probe.py -- does the NUMA node of a host image, and where the
staging lanes / copy threads sit, set the rate of the host paths (config 5)?

The GPU hangs off one socket's PCIe root; a page-locked image whose pages sit
on the other socket's memory is DMA'd across the inter-socket link, and the
staged path's copy threads read the image and write the lanes.  For every
NUMA node: a GiB-sized image first-touched by threads pinned to that node's
CPUs (first touch places the pages), then
  * bt_sha1_chunks_host on the image unregistered (staged through the
    library's pinned lanes): median of `reps` runs after a first one, with
    the pipeline's phase split and placement (bt_sha1_get_pipeline_stats);
  * the same on the registered image (direct DMA, 2 streams);
  * raw H2D of the registered image (hipMemcpy through torch).
Prints one JSON line per node.  The staging placement is the library's
(BT_SHA1_NUMA=gpu, the default: lanes on the GPU's node, copy threads on its
CPUs; BT_SHA1_NUMA=off: neither), BT_SHA1_COPY_THREADS the copy thread
count, BT_SHA1_COPY_ORDER the H2D order -- run the probe once per setting.
usage: numa_probe.py [GiB] [reps]
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


def runs(fn, gib, reps, stats=False):
    """First run, then `reps` more: median / min / max GiB/s of the latter,
    and the phase split of the median run."""
    rows = []
    for _ in range(1 + reps):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        row = {"GiB_per_s": round(gib / dt, 3)}
        if stats:
            s = bt.pipeline_stats()
            row.update(fill_s=s["fill_s"], wait_s=s["wait_s"], s=round(dt, 4))
        rows.append(row)
    steady = sorted(rows[1:], key=lambda r: r["GiB_per_s"])
    out = {"median": steady[len(steady) // 2]["GiB_per_s"], "min": steady[0]["GiB_per_s"],
           "max": steady[-1]["GiB_per_s"], "first": rows[0]["GiB_per_s"]}
    if stats:
        out["median_run"] = steady[len(steady) // 2]
    return out


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
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
        staged = runs(lambda: bt.chunks_host_addr(addr, nbytes), gib, reps, stats=True)
        st = bt.pipeline_stats()
        bt.host_register(addr, nbytes)
        try:
            direct = runs(lambda: bt.chunks_host_addr(addr, nbytes), gib, reps)
            src = torch.from_numpy(img)

            def h2d():
                scratch.copy_(src, non_blocking=True)
                torch.cuda.synchronize()
            raw = runs(h2d, gib, 3)
        finally:
            bt.host_unregister(addr)
        print(json.dumps({"image_node": node, "gpu": bdf, "gpu_node": gnode, "GiB": round(nbytes / 2**30, 2),
                          "numa_env": os.environ.get("BT_SHA1_NUMA", "default"),
                          "copy_threads": st["copy_threads"], "policy": st["numa_policy"],
                          "image_pages": st["src_pages"], "lane_pages": st["lane_pages"],
                          "copy_pieces": st["copy_pieces"],
                          "raw_h2d_registered": raw, "chunks_host_registered": direct,
                          "chunks_host_staged": staged}), flush=True)
        del img


if __name__ == "__main__":
    main()
