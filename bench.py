#!/usr/bin/env python3
"""bench.py -- device-resident SHA-1 chunk hashing on MI355X (BASELINE.json metric).

Workload (BASELINE config 3 per GPU, config 4 across GPUs): every rank holds
`--chunks` (default 131072) synthetic 512 KiB chunks = 64 GiB resident in its
HBM, generated in place by the frozen counter-based generator with GLOBAL
chunk indices [rank*C, (rank+1)*C) (so N=8 is exactly config 4's 1 M chunks).
One step = one launch of the hot kernel over all of the rank's chunks -> 20 B
digests in HBM.  Weak scaling, no data-path collective: ranks only meet at the
timing barriers, the max-over-ranks reduction, and a host-side (gloo) gather
of digests after the timed region.

Timed region: W untimed warmup steps, then barrier + synchronize, K steps,
synchronize + barrier; value = all ranks' chunk bytes * K / max-over-ranks
wall time, in GiB/s.  The hot kernel's own duration is also taken live with
HIP events on the stream it is launched on (torch's current stream), for the
roofline.  rank 0 at N=1 additionally times the reference sha.c
(oracle/_ref/libref_sha1.so, compiled from the reference) on the host cores
over a bounded sample of the same chunks, and cross-checks those digests.
"""
import argparse
import ctypes
import importlib.util
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "bittorrent-with-congestion-control_amd")
CHUNK = 512 * 1024
SEED = 0x0B175EED
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
VALU_OPS_PER_BLOCK = 597       # counted in the kernel's ISA
VALU_HALF_RATE_PER_BLOCK = 400  # v_alignbit / v_add3 / v_perm: 16 lanes/clk/SIMD (tools/ubench)
VALU_FULL_RATE_PER_BLOCK = 197  # v_bitop3 / v_xor / v_add: 32 lanes/clk/SIMD with co-issue
SIMDS, CLOCK_GHZ = 1024, 2.4
# VALU ceiling for this exact instruction mix: a wave64 half-rate op holds the
# SIMD 4 clocks, a full-rate op 2 -> 1994 clocks per 64-byte block per wave.
_MIX_CLK = 4 * VALU_HALF_RATE_PER_BLOCK + 2 * VALU_FULL_RATE_PER_BLOCK
VALU_MIX_PEAK_TOPS = VALU_OPS_PER_BLOCK * 64 * SIMDS * CLOCK_GHZ * 1e9 / _MIX_CLK / 1e12  # lane-ops/s, ~47.1


def load_btsha1():
    if not os.path.exists(os.path.join(PKG, "libbtsha1.so")):  # clean checkout: build once
        import fcntl
        import subprocess
        with open(os.path.join(HERE, ".build.lock"), "w") as lk:  # N ranks start together
            fcntl.flock(lk, fcntl.LOCK_EX)
            if not os.path.exists(os.path.join(PKG, "libbtsha1.so")):
                subprocess.run(["make", "-C", HERE, "lib"], check=True)
    spec = importlib.util.spec_from_file_location("btsha1", os.path.join(PKG, "btsha1.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(host, n_chunks, gpu_digests, want_threads):
    """Reference sha.c (or, if its prebuilt .so is absent, our port) on host cores."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import py_oracle
    ref = py_oracle.load_reference("O2")
    kind, flags = ("reference", "-O2 (reference chunk.c + sha.c)") if ref is not None else \
        ("port", "-O2 (oracle/sha1_oracle.c)")
    import numpy as np
    base = host.ctypes.data
    out = (ctypes.c_uint8 * (20 * n_chunks))()

    def hash_range(lo, hi):
        for i in range(lo, hi):
            if ref is not None:
                ref.shahash(ctypes.c_void_p(base + i * CHUNK), CHUNK, ctypes.byref(out, 20 * i))
            else:
                py_oracle._lib.or_shahash(ctypes.c_void_p(base + i * CHUNK), CHUNK, ctypes.byref(out, 20 * i))

    def run(threads, n):
        ts = [threading.Thread(target=hash_range, args=(n * t // threads, n * (t + 1) // threads))
              for t in range(threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return time.perf_counter() - t0

    n1 = min(n_chunks, 2048)  # ~1.5 s on one core
    t1 = run(1, n1)
    tn = run(want_threads, n_chunks)
    ok = bytes(out) == gpu_digests[:20 * n_chunks]
    gib = n_chunks * CHUNK / 2**30
    o0 = None  # the reference Makefile's own flags (-g, no -O): 1 thread, 256 chunks
    ref0 = py_oracle.load_reference("O0")
    if ref0 is not None:
        n0 = min(n_chunks, 256)
        o0_out = (ctypes.c_uint8 * 20)()
        t0 = time.perf_counter()
        for i in range(n0):
            ref0.shahash(ctypes.c_void_p(base + i * CHUNK), CHUNK, o0_out)
        o0 = round(n0 * CHUNK / 2**30 / (time.perf_counter() - t0), 4)
    return {
        "value": round(gib / tn, 4), "unit": "GiB/s", "cores": want_threads, "kind": kind,
        "sample": f"{n_chunks} x 512 KiB chunks ({gib:.1f} GiB) of the same synthetic workload, "
                  f"shahash per chunk, {want_threads} threads; 1 thread: "
                  f"{round(n1 * CHUNK / 2**30 / t1, 4)} GiB/s",
        "flags": flags, "digests_match_gpu": ok, "reference_O0_1thread_GiBs": o0,
        "host_cpu": _cpu_model(),
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chunks", type=int, default=131072, help="512 KiB chunks per GPU")
    ap.add_argument("--ring", type=int, default=0, help="kernel ring depth (0 = library default)")
    ap.add_argument("--lines", type=int, default=1, help="128-byte lines per ring slot (with --ring)")
    ap.add_argument("--nt", type=int, default=0, help="non-temporal loads (with --ring)")
    ap.add_argument("--pitch", type=int, default=CHUNK, help="bytes between chunk starts in HBM")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-chunks", type=int, default=32768,
                    help="CPU-baseline sample: 16 GiB, ~25 core-seconds of reference sha.c")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL; gloo for rehearsals)")
    ap.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "traffic_r01.json"))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())  # == local on a full node
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            cpu_group = dist.new_group(backend="gloo")
        else:
            dist.init_process_group(args.backend)
            cpu_group = None
    bt = load_btsha1()
    if args.ring:
        bt.set_variant(args.ring, args.lines, args.nt)

    C = args.chunks
    pitch = args.pitch
    buf = torch.empty(pitch * (C - 1) + CHUNK + 256, dtype=torch.uint8, device="cuda")
    dig = torch.zeros(20 * C, dtype=torch.uint8, device="cuda")
    # A dedicated stream (torch's default stream has handle 0, which the C-ABI
    # reads as "library stream"): kernels and timing events share it.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp != 0
    first_chunk = rank * C
    if pitch == CHUNK:
        bt.fill_synthetic(buf.data_ptr(), C * CHUNK, first_chunk * (CHUNK // 8), SEED, sp)
    else:  # padded layout: fill chunk by chunk (same bytes per chunk)
        for i in range(C):
            bt.fill_synthetic(buf.data_ptr() + i * pitch, CHUNK, (first_chunk + i) * (CHUNK // 8), SEED, sp)
    torch.cuda.synchronize()

    def step():
        bt.chunks_dev(buf.data_ptr(), C, CHUNK, pitch, dig.data_ptr(), sp)

    for _ in range(args.warmup):
        step()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)

    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device="cuda" if args.backend == "nccl" else "cpu")
    per_rank = [t.clone() for _ in range(world)]
    if world > 1:
        dist.all_gather(per_rank, t)  # config 4 wants per-GPU rates beside the aggregate
    per_rank = [(float(x[0]), float(x[1])) for x in per_rank]
    wall_max = max(w for w, _ in per_rank)
    kern_max = max(k for _, k in per_rank)

    # Host-side gather of digests (after timing): rank order == global chunk order.
    host_dig = dig.cpu()
    if world > 1:
        parts = [torch.empty_like(host_dig) for _ in range(world)] if rank == 0 else None
        dist.gather(host_dig, parts, dst=0, group=cpu_group)
        all_dig = torch.cat(parts).numpy().tobytes() if rank == 0 else None
    else:
        all_dig = host_dig.numpy().tobytes()

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    total_bytes = world * C * CHUNK * args.steps
    value = total_bytes / wall_max / 2**30
    bytes_per_launch = C * CHUNK
    achieved = bytes_per_launch / (kern_max * 1e-3) / 1e9
    # one lane-op per instruction per chunk-lane
    valu_tops = C * (CHUNK // 64 + 1) * VALU_OPS_PER_BLOCK / (kern_max * 1e-3) / 1e12

    # Parity spot check of the timed output: global chunks 0..4095 are the
    # committed golden vectors (tests/golden/synth4096.txt, from sha.c).
    parity = None
    golden = os.path.join(HERE, "tests", "golden", "synth4096.txt")
    if os.path.exists(golden) and C >= 4096:
        rows = [l.split() for l in open(golden) if not l.startswith("#")]
        parity = all(all_dig[20 * int(i):20 * int(i) + 20].hex() == h for i, h in rows)

    traffic = None
    traffic_src = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("chunks") == C and tj.get("pitch", CHUNK) == pitch:
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(args.traffic_json, HERE)
        except (OSError, ValueError):
            pass

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        n = min(args.cpu_chunks, C)
        import numpy as np
        host = np.empty(n * CHUNK, dtype=np.uint8)
        if pitch == CHUNK:
            step = 2048 * CHUNK  # 1 GiB slices: no second full-size host copy
            for o in range(0, n * CHUNK, step):
                host[o:o + step] = buf[o:min(o + step, n * CHUNK)].cpu().numpy()
        else:
            for i in range(n):
                host[i * CHUNK:(i + 1) * CHUNK] = buf[i * pitch:i * pitch + CHUNK].cpu().numpy()
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        cpu = cpu_baseline(host, n, all_dig, threads)

    line = {
        "metric": "GiB/s SHA-1 hashed (device-resident 512KiB chunks) at 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: device-generated splitmix64 stream (seed 0x0B175EED, global chunk index)",
        "config": {
            "workload": f"{C} x 512 KiB chunks per GPU, device-resident ({C * CHUNK / 2**30:.0f} GiB/GPU), "
                        "one hot-kernel launch per step -> 20 B digests",
            "chunks_per_gpu": C, "chunk_bytes": CHUNK, "pitch_bytes": pitch,
            "global_chunks": world * C,
            "parallelism": f"dp{world} (contiguous chunk-range split, no data-path collective)",
            "kernel_variant": bt.build_info().split("hip")[-1].split(" ", 1)[-1],
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "k_sha1_fixed", "kernel_ms": round(kern_max, 4),
            "algorithmic_bytes_per_launch": bytes_per_launch, "traffic_source": traffic_src,
        },
        "valu_roofline": {"bound": "valu", "achieved": round(valu_tops, 2), "peak": round(VALU_MIX_PEAK_TOPS, 2),
                          "unit": "T int32 lane-ops/s", "frac": round(valu_tops / VALU_MIX_PEAK_TOPS, 4),
                          "ops_per_block": VALU_OPS_PER_BLOCK,
                          "peak_basis": f"{VALU_OPS_PER_BLOCK}-instruction mix ({VALU_HALF_RATE_PER_BLOCK} half-rate, "
                                        f"{VALU_FULL_RATE_PER_BLOCK} full-rate) at 2.4 GHz on 1024 SIMDs"},
        "per_gpu": [{"rank": r, "GiB_per_s": round(C * CHUNK * args.steps / w / 2**30, 3),
                     "kernel_ms": round(k, 4)} for r, (w, k) in enumerate(per_rank)],
        "parity_first_4096_vs_golden": parity,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
