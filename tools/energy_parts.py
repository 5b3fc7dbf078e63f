#!/usr/bin/env python3
"""tools/energy_parts.py -- where the hot kernel's energy goes.

Runs each workload as a CHILD process (this process never touches HIP; it only
reads the SMU through amdsmi) and, while it runs, samples the energy
accumulator, the limiter residency counters and the per-XCD gfx clocks every
50 ms.  Power = delta energy / delta time over the middle of the child's busy
period (the first 30 % and last 10 % are dropped: ramp-up and tail).  Each
workload prints its own rate; energy per GiB = power / rate.

  idle      nothing running
  hbm       the production k_sha1_fixed over 131072 x 512 KiB chunks in HBM
  mall      the same kernel and grid, chunks overlapping in a ~128 MiB footprint
  l2        the same kernel and grid, all lanes on the same ~2.5 MiB
  alu       the SHA-1 compression alone, no memory traffic (sha1_alu long)
  stream    a read-only stream in the hot kernel's per-lane pattern
  coalesced a read-only stream, 8 lines per wave instruction

One JSON line per case.  usage: energy_parts.py [seconds per case] [grouped]
(`grouped`: only the read-only streams with G = 1, 2, 4, 8 lanes per line)
"""
import json
import os
import re
import statistics
import subprocess
import sys
import threading
import time

import amdsmi

HERE = os.path.dirname(os.path.abspath(__file__))
UB = os.path.join(HERE, "ubench")


def handle():
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    return hs[int(vis.split(",")[0])] if vis and len(hs) > 1 else hs[0]


def sample(h):
    m = amdsmi.amdsmi_get_gpu_metrics_info(h)
    e = amdsmi.amdsmi_get_energy_count(h)
    clks = [c for c in m.get("current_gfxclks", []) if isinstance(c, (int, float))]
    return {"t": time.perf_counter(), "J": e["energy_accumulator"] * e["counter_resolution"] * 1e-6,
            "W": m.get("current_socket_power"), "clk": statistics.median(clks) if clks else None,
            "ppt": m.get("ppt_residency_acc"), "acc": m.get("accumulation_counter")}


def measure(h, cmd, seconds):
    samples, stop = [], threading.Event()

    def loop():
        while not stop.is_set():
            samples.append(sample(h))
            stop.wait(0.05)

    th = threading.Thread(target=loop, daemon=True)
    th.start()
    out = ""
    if cmd:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        out = r.stdout + r.stderr
        if r.returncode:
            raise SystemExit(f"{cmd}: rc={r.returncode}\n{out}")
    else:
        time.sleep(seconds)
    stop.set()
    th.join()
    busy = [s for s in samples if not cmd or (s["W"] or 0) > 500]
    if len(busy) < 8:
        busy = samples
    t0, t1 = busy[0]["t"], busy[-1]["t"]
    win = [s for s in busy if t0 + 0.3 * (t1 - t0) <= s["t"] <= t1 - 0.1 * (t1 - t0)]
    a, b = win[0], win[-1]
    watts = (b["J"] - a["J"]) / (b["t"] - a["t"])
    ppt = (b["ppt"] - a["ppt"]) / (b["acc"] - a["acc"]) if b["acc"] != a["acc"] else None
    return watts, statistics.median(s["clk"] for s in win if s["clk"]), ppt, b["t"] - a["t"], out


def rate_gib(out):
    m = re.search(r"([\d.]+) GiB/s hashed", out)
    if m:
        return float(m.group(1))
    m = re.search(r"([\d.]+) GB/s", out)
    return float(m.group(1)) * 1e9 / 2**30 if m else None


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    h = handle()
    n_launch = int(secs * 1000 / 19)  # ~19 ms per launch at 131072 chunks
    cases = [
        ("idle", None),
        ("hbm", [os.path.join(UB, "residency"), "131072", str(n_launch), "1", "0"]),
        ("mall", [os.path.join(UB, "residency"), "131072", str(n_launch), "1", "1"]),
        ("l2", [os.path.join(UB, "residency"), "131072", str(n_launch), "1", "2"]),
        ("alu", [os.path.join(UB, "sha1_alu"), "long", str(int(secs * 1000 / 8.5))]),
        ("stream", [os.path.join(UB, "streamread"), str(int(secs * 1000 / 17)), "0"]),
        ("coalesced", [os.path.join(UB, "streamread"), str(int(secs * 1000 / 11)), "2"]),
    ]
    if len(sys.argv) > 2 and sys.argv[2] == "grouped":  # read patterns only
        cases = [cases[0]] + [(f"stream_g{g}", [os.path.join(UB, "streamread"), str(int(secs * 1000 / 15)), str(m)])
                              for g, m in ((1, 0), (2, 4), (4, 5), (8, 6), (1, 0))]
    idle = None
    for name, cmd in cases:
        watts, clk, ppt, win_s, out = measure(h, cmd, secs)
        if name == "idle":
            idle = watts
        rate = rate_gib(out) if cmd else None
        row = {"case": name, "socket_W": round(watts, 1), "gfxclk_MHz": clk, "ppt_residency": None if ppt is None
               else round(ppt, 3), "window_s": round(win_s, 2), "GiB_per_s": rate}
        if rate:
            row["J_per_GiB"] = round(watts / rate, 4)
            row["J_per_GiB_above_idle"] = round((watts - idle) / rate, 4)
        print(json.dumps(row), flush=True)
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
