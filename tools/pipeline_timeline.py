#!/usr/bin/env python3
"""tools/pipeline_timeline.py -- where the time of one host pipeline call goes,
for a kernel + copy trace (run it under `rocprofv3 --kernel-trace
--memory-copy-trace --output-format csv`).

An 8 GiB pageable image (bench.py's host leg, written by numpy) is hashed
with bt_sha1_chunks_host `calls` times; each call's wall interval is printed
(perf_counter and, for matching against the trace, CLOCK_MONOTONIC ns, the
clock rocprofv3 stamps with) beside the library's pipeline stats.  With
`--summary DIR` instead, reads the trace CSVs rocprofv3 wrote under DIR and
prints, per call: the copies (b = a lane batch, c = a column of the split
tail), the gaps between them, and the kernels still running after the last.
usage: pipeline_timeline.py [calls] [GiB]  |  pipeline_timeline.py --summary DIR
"""
import csv
import glob
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(calls, gib):
    import numpy as np
    import torch  # noqa: F401  (the HIP runtime first)
    sys.path.insert(0, os.path.join(HERE, "bittorrent-with-congestion-control_amd"))
    import btsha1 as bt

    n = int(gib * 2048)
    img = np.empty(n * 524288, dtype=np.uint8)
    img.view(np.uint64)[:] = np.arange(img.size // 8, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    ref = None
    for i in range(calls):
        t0, m0 = time.perf_counter(), time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        got = bt.chunks_host_addr(img.ctypes.data, img.nbytes)
        t1, m1 = time.perf_counter(), time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        st = bt.pipeline_stats()
        ref = got if ref is None else ref
        print(json.dumps({"call": i, "s": round(t1 - t0, 4), "GiB_per_s": round(img.nbytes / (t1 - t0) / 2**30, 2),
                          "mono_ns": [m0, m1], "same_digests": got == ref,
                          **{k: st[k] for k in ("feed", "batches", "batch_bytes", "column_chunks", "wait_s",
                                                "register_s", "unregister_s")}}), flush=True)


def summary(d):
    def rows(pattern):
        out = []
        for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
            with open(f) as fh:
                out += list(csv.DictReader(fh))
        return out

    kern = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40])
                   for r in rows("*kernel_trace.csv")), key=lambda x: x[0])
    copies = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", ""))
                     for r in rows("*memory_copy_trace.csv")), key=lambda x: x[0])
    # the trace carries no byte counts: the pipeline's batch copies are the H2D
    # ones over 1 ms; the column-split tail's strided copies out of locked host
    # pages are traced as DEVICE_TO_DEVICE (the runtime sees a device-mapped
    # source) -- "column" in copy_kinds
    big = [c for c in copies if ("HOST_TO_DEVICE" in c[2] or "DEVICE_TO_DEVICE" in c[2]) and c[1] - c[0] > 1_000_000]
    # calls: runs of copies separated by > 0.5 ms (within a call they are back to back)
    groups, cur = [], []
    for c in big:
        if cur and c[0] - cur[-1][1] > 500_000:
            groups.append(cur)
            cur = []
        cur.append(c)
    if cur:
        groups.append(cur)
    for gi, g in enumerate(groups):
        c0, c1 = g[0][0], g[-1][1]
        nxt = groups[gi + 1][0][0] if gi + 1 < len(groups) else c1 + 100_000_000
        after = [k for k in kern if c0 <= k[1] and k[0] < nxt]
        tail = [k for k in after if k[1] > c1]
        end = max([c1] + [k[1] for k in tail])
        line = {"call": gi, "copies": len(g), "copy_span_ms": round((c1 - c0) / 1e6, 3),
                "copy_gaps_ms": [round((g[i + 1][0] - g[i][1]) / 1e6, 3) for i in range(len(g) - 1)],
                "copy_ms": [round((c[1] - c[0]) / 1e6, 3) for c in g],
                "copy_kinds": "".join("c" if "DEVICE_TO_DEVICE" in c[2] else "b" for c in g),
                "end_after_last_copy_ms": round((end - c1) / 1e6, 3),
                "tail_kernels": [{"name": k[2], "start_ms": round((k[0] - c1) / 1e6, 3),
                                  "dur_ms": round((k[1] - k[0]) / 1e6, 3)} for k in tail],
                "kernels_during_copies": len(after) - len(tail)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 4, float(sys.argv[2]) if len(sys.argv) > 2 else 8)
