#!/usr/bin/env python3
"""tools/traffic_json.py -- the hot kernel's HBM traffic per launch from the
rocprofv3 --pmc passes of `tools/gpu_session.sh pmc`, as the
profiles/traffic_rNN.json bench.py's roofline.traffic cites.

Reads every *counter_collection.csv under DIR (one row per dispatch and
counter), keeps the dispatches of the hot kernel (k_sha1_fixed), averages
each counter over them and applies MI355X_MICROARCH.md's gfx950 reading:
FETCH_SIZE is in KiB and counts half the bytes of a wide coalesced read
(x1024 x2); TCC_EA0_RDREQ counts 128-byte requests (x128, plus x32 for the
32-byte ones).  The file is keyed on what bench.py checks before using it:
the library's source id and variant (read from the built library), the
kernel, and the layout (131072 chunks at a 512 KiB pitch, bench.py's
default).  Also writes the per-counter means to SUMMARY.
usage: traffic_json.py DIR OUT.json [SUMMARY.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHUNKS, PITCH = 131072, 524288


def main():
    d, out = sys.argv[1], sys.argv[2]
    summary_path = sys.argv[3] if len(sys.argv) > 3 else None
    vals = defaultdict(list)
    kms = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            if "k_sha1_fixed" not in r.get("Kernel_Name", ""):
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (f, r.get("Dispatch_Id"))
            if key not in seen and r.get("Start_Timestamp") and r.get("End_Timestamp"):
                seen.add(key)
                kms.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    if not vals:
        sys.exit(f"no k_sha1_fixed dispatches under {d}")
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    summary = dict(mean, profiled_dispatches=len(kms), profiled_kernel_ms_mean=sum(kms) / len(kms) if kms else None)
    sys.path.insert(0, os.path.join(HERE, "bittorrent-with-congestion-control_amd"))
    import btsha1 as bt
    algo = CHUNKS * PITCH
    fetch = mean["FETCH_SIZE"] * 1024 * 2 if "FETCH_SIZE" in mean else None
    rdreq = (mean["TCC_EA0_RDREQ_sum"] * 128 + mean.get("TCC_EA0_RDREQ_32B_sum", 0.0) * 32
             if "TCC_EA0_RDREQ_sum" in mean else None)
    hbm = fetch if fetch is not None else rdreq
    tj = {"chunks": CHUNKS, "pitch": PITCH, "hbm_bytes_per_launch": hbm, "source_id": bt.source_id(),
          "variant": bt.build_info().split("ring=")[1].split()[0], "kernel": "k_sha1_fixed",
          "algorithmic_bytes_per_launch": algo, "ratio": hbm / algo if hbm else None,
          "fetch_size_bytes_corrected": fetch, "rdreq_bytes": rdreq,
          "method": "rocprofv3 --pmc FETCH_SIZE (x1024 KiB, x2 gfx950 half-count) and TCC_EA0_RDREQ_sum x128 B, "
                    "separate passes, hot kernel dispatches averaged (tools/traffic_json.py)"}
    json.dump(tj, open(out, "w"), indent=1)
    print(json.dumps(tj))
    if summary_path:
        json.dump(summary, open(summary_path, "w"), indent=1)


if __name__ == "__main__":
    main()
