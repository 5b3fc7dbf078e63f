#!/usr/bin/env python3
"""Turn the rocprofv3 CSVs of a gpu_session `prof` + `pmc` run into the
committed evidence under profiles/<round>/:

  kernel_stats.csv         rocprofv3 --kernel-trace --stats summary (copied)
  pmc_summary.json         per-dispatch counters of the hot kernel, averaged
  summary.md               human-readable table
  ../traffic_<round>.json  HBM bytes per launch for bench.py's roofline.traffic

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and on gfx950
reports half of a wide streaming read, so bytes = FETCH_SIZE * 1024 * 2; the
memory-side request count TCC_EA0_RDREQ_sum (128-byte requests here, with
TCC_EA0_RDREQ_32B_sum = 0) gives the same figure independently.
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

HOT = "k_sha1_fixed<3, 1, 0, false, false>"  # the production instantiation (not the stamped probe build)


def counters(path):
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    meta = {}
    for r in csv.DictReader(open(path)):
        if HOT not in r["Kernel_Name"]:
            continue
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Grid_Size"], r.get("VGPR_Count"))
    return per, meta


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
    chunks = int(sys.argv[3]) if len(sys.argv) > 3 else 131072
    out = os.path.join("profiles", rnd)
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, "prof", "bench_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copyfile(stats, os.path.join(out, "kernel_stats.csv"))
    agg = defaultdict(list)
    durs = []
    for name in ("fetch", "rdreq", "valu", "valu2", "wait"):
        p = os.path.join(src, "pmc", f"{name}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        per, meta = counters(p)
        for d, cs in per.items():
            for k, v in cs.items():
                agg[k].append(v)
            durs.append((meta[d][1] - meta[d][0]) * 1e-6)
    # The bench line printed by the profiled process itself (gpu_session `prof`).
    bench_line = None
    pl = os.path.join(src, "prof.log")
    if os.path.exists(pl):
        for l in open(pl):
            if l.startswith("{") and '"metric"' in l:
                bench_line = json.loads(l)
    if bench_line:
        json.dump(bench_line, open(os.path.join(out, "bench_line_same_process.json"), "w"), indent=1)
    summary = {k: statistics.mean(v) for k, v in agg.items()}
    summary["profiled_dispatches"] = len(durs)
    summary["profiled_kernel_ms_mean"] = statistics.mean(durs) if durs else None
    algo = chunks * 512 * 1024
    traffic = {}
    if "FETCH_SIZE" in summary:
        traffic["fetch_size_bytes_corrected"] = summary["FETCH_SIZE"] * 1024 * 2
    if "TCC_EA0_RDREQ_sum" in summary:
        traffic["rdreq_bytes"] = summary["TCC_EA0_RDREQ_sum"] * 128 + summary.get("TCC_EA0_RDREQ_32B_sum", 0) * 32
    json.dump(summary, open(os.path.join(out, "pmc_summary.json"), "w"), indent=1)
    if traffic:
        hbm = traffic.get("fetch_size_bytes_corrected", traffic.get("rdreq_bytes"))
        build = (bench_line or {}).get("config", {}).get("build", "")
        tj = {"chunks": chunks, "pitch": 512 * 1024, "hbm_bytes_per_launch": hbm,
              "source_id": build.split("src=")[1].split()[0] if "src=" in build else None,
              "variant": build.split("ring=")[1].split()[0] if "ring=" in build else None,
              "kernel": "k_sha1_fixed",
              "algorithmic_bytes_per_launch": algo, "ratio": hbm / algo, **traffic,
              "method": "rocprofv3 --pmc FETCH_SIZE (x1024 KiB, x2 gfx950 half-count) and TCC_EA0_RDREQ_sum x128 B, "
                        "separate passes, hot kernel dispatches averaged"}
        json.dump(tj, open(os.path.join("profiles", f"traffic_{rnd}.json"), "w"), indent=1)
    lines = [f"# Profile summary {rnd}", "", f"hot kernel `{HOT}`, {chunks} x 512 KiB chunks per launch", ""]
    if os.path.exists(stats):
        lines += ["## rocprofv3 --kernel-trace --stats", "", "| kernel | calls | avg ms | min ms | max ms |", "|---|---|---|---|---|"]
        hot_avg = None
        for r in csv.DictReader(open(stats)):
            lines.append(f"| {r['Name'][:70]} | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
                         f"{float(r['MinNs'])/1e6:.3f} | {float(r['MaxNs'])/1e6:.3f} |")
            if HOT in r["Name"]:
                hot_avg = float(r["AverageNs"]) / 1e6
        lines.append("")
        # The timed launches alone: the last `steps` hot-kernel dispatches of the trace.
        trace = os.path.join(src, "prof", "bench_kernel_trace.csv")
        timed_avg = None
        if bench_line and os.path.exists(trace):
            d = sorted((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
                       for r in csv.DictReader(open(trace)) if HOT in r["Kernel_Name"])
            last = [ms for _, ms in d[-bench_line["steps"]:]]
            timed_avg = statistics.mean(last) if last else None
        if bench_line and hot_avg:
            rf = bench_line["roofline"]
            frac_prof = algo / (hot_avg * 1e-3) / 1e9 / rf["peak"]

            lines += ["## Same process: bench line vs rocprof", "",
                      f"bench (HIP events, {bench_line['steps']} timed launches): kernel {rf['kernel_ms']:.3f} ms, "
                      f"frac {rf['frac']:.4f}; ms_per_step {bench_line['ms_per_step']:.3f}; value {bench_line['value']} GiB/s",
                      f"rocprof average over all launches of the same process: {hot_avg:.3f} ms -> frac "
                      f"{frac_prof:.4f} ({100 * (frac_prof / rf['frac'] - 1):+.2f} % vs the bench line)",
                      f"build: {bench_line['config'].get('build')}", ""]
            if timed_avg:
                frac_timed = algo / (timed_avg * 1e-3) / 1e9 / rf["peak"]
                lines[-1:-1] = [f"rocprof trace, the {bench_line['steps']} timed launches only: {timed_avg:.3f} ms -> "
                                f"frac {frac_timed:.4f} ({100 * (frac_timed / rf['frac'] - 1):+.2f} % vs the bench line)"]
    if summary:
        lines += ["## PMC (hot kernel, mean per dispatch)", "", "| counter | value |", "|---|---|"]
        for k, v in sorted(summary.items()):
            lines.append(f"| {k} | {v:.6g} |" if isinstance(v, float) else f"| {k} | {v} |")
        lines.append("")
    if traffic:
        lines += [f"HBM read bytes per launch: {hbm:.4g} (algorithmic {algo:.4g}, ratio {hbm/algo:.3f})", ""]
    open(os.path.join(out, "summary.md"), "w").write("\n".join(lines))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
