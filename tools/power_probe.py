#!/usr/bin/env python3
"""Which limiter sets the hot kernel's clock?  Runs the BASELINE step
(131072 x 512 KiB chunks, k_sha1_fixed) back to back for `seconds` and prints,
as JSON lines, the full amdsmi gpu_metrics before and after, the deltas of its
accumulators (residency counters of the power / thermal / current limiters,
energy), and samples of power, clocks and temperatures every 100 ms.

usage: power_probe.py [seconds] [chunks]
"""
import importlib.util
import json
import os
import sys
import threading
import time

import torch

import amdsmi

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHUNK = 512 * 1024


def load_bt():
    spec = importlib.util.spec_from_file_location(
        "btsha1", os.path.join(HERE, "bittorrent-with-congestion-control_amd", "btsha1.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def handle():
    amdsmi.amdsmi_init()
    p = torch.cuda.get_device_properties(0)
    want = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    for h in amdsmi.amdsmi_get_processor_handles():
        dom, bus, rest = amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")
        if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
            return h
    raise SystemExit("no amdsmi handle for cuda:0")


def scalar_items(m):
    return {k: v for k, v in m.items() if isinstance(v, (int, float))}


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
    bt = load_bt()
    h = handle()
    buf = torch.empty(n * CHUNK + 256, dtype=torch.uint8, device="cuda")
    dig = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    bt.fill_synthetic(buf.data_ptr(), n * CHUNK, 0, 0x0B175EED, s)
    torch.cuda.synchronize()
    time.sleep(1.0)
    m0 = amdsmi.amdsmi_get_gpu_metrics_info(h)
    print(json.dumps({"metrics_idle": m0}, default=str), flush=True)
    samples, stop = [], threading.Event()

    def sampler():
        t0 = time.perf_counter()
        while not stop.is_set():
            try:
                m = amdsmi.amdsmi_get_gpu_metrics_info(h)
                samples.append({"t": round(time.perf_counter() - t0, 3), "W": m.get("current_socket_power"),
                                "gfxclks": m.get("current_gfxclks"), "uclk": m.get("current_uclk"),
                                "fclk": m.get("current_fclk"), "hot": m.get("temperature_hotspot"),
                                "mem": m.get("temperature_mem"), "vrgfx": m.get("temperature_vrgfx"),
                                "throttle": m.get("throttle_status"), "indep": m.get("indep_throttle_status")})
            except Exception as e:  # noqa: BLE001
                samples.append({"err": str(e)})
            stop.wait(0.1)

    ma = amdsmi.amdsmi_get_gpu_metrics_info(h)
    t0 = time.perf_counter()
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    launches = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(10):
            bt.chunks_dev(buf.data_ptr(), n, CHUNK, CHUNK, dig.data_ptr(), s)
        launches += 10
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    mb = amdsmi.amdsmi_get_gpu_metrics_info(h)
    stop.set()
    th.join()
    a, b = scalar_items(ma), scalar_items(mb)
    print(json.dumps({"launches": launches, "seconds": round(dt, 3),
                      "GiB_per_s": round(launches * n * CHUNK / dt / 2**30, 2)}), flush=True)
    print(json.dumps({"deltas": {k: b[k] - a[k] for k in sorted(a) if k in b and b[k] != a[k]}}), flush=True)
    print(json.dumps({"metrics_end": mb}, default=str), flush=True)
    for r in samples:
        print(json.dumps(r), flush=True)
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
