#!/usr/bin/env python3
"""bench.py -- device-resident SHA-1 chunk hashing on MI355X (BASELINE.json metric).

Workload (BASELINE config 3 per GPU, config 4 across GPUs): every rank holds
`--chunks` (default 131072) synthetic 512 KiB chunks = 64 GiB resident in its
HBM, generated in place by the frozen counter-based generator with GLOBAL
chunk indices [rank*C, (rank+1)*C) (so N=8 is exactly config 4's 1 M chunks).
One step = one launch of the hot kernel over all of the rank's chunks -> 20 B
digests in HBM.  Weak scaling, no data-path collective: ranks only meet on a
CPU (gloo) group for the timing barriers, the max-over-ranks reduction and a
host-side gather of digests after the timed region (shard.run_rank).

Timed region: W untimed warmup steps, then barrier + synchronize, K steps,
synchronize + barrier; value = all ranks' chunk bytes * K / max-over-ranks
wall time, in GiB/s.  The hot kernel's own duration is also taken live with
HIP events on the stream it is launched on, for the roofline.

After the timed region:
  * every rank: the in-kernel shader clock of the hot kernel (stamped
    diagnostic build, bt_sha1_clock_probe), so the VALU roofline is priced
    at the clock the chip actually held as well as at the nominal 2.4 GHz;
  * every rank, all together: `power`, the socket power of its GPU from the
    SMU energy accumulator while the timed step runs back to back for
    --power-s seconds, against the board's power cap (the bound that sets
    the hot kernel's clock);
  * rank 0 at every N (the other ranks wait at the final barrier):
    cpu_baseline, the reference sha.c (oracle/_ref, compiled from the
    reference) or our restatement (oracle/, "port") on the host cores, 4096
    of rank 0's chunks at 1 thread and at every core this process may use,
    at -O2 and at the reference Makefile's -O0;
  * rank 0 at N=1: verify_dev (the fused compare, paired with the hash) and
    host_path, config 5's PCIe-inclusive host->digest rates of the pipelines
    that start in host memory (never `value`): median of 5 steady runs with
    each run's phase split, NUMA placement and cgroup throttling, and the
    batched verifier fed zero-copy and packetized (util.c:275).
"""
import argparse
import ctypes
import glob
import importlib.util
import json
import math
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time

_T_IMPORT = time.perf_counter()

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "bittorrent-with-congestion-control_amd")
CHUNK = 512 * 1024
SEED = 0x0B175EED
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
VALU_OPS_PER_BLOCK = 597       # counted in the kernel's ISA (tests/test_isa.py)
VALU_HALF_RATE_PER_BLOCK = 400  # v_alignbit / v_add3 / v_perm: 16 lanes/clk/SIMD (tools/ubench)
VALU_FULL_RATE_PER_BLOCK = 197  # v_bitop3 / v_xor / v_add: 32 lanes/clk/SIMD
SIMDS, CLOCK_GHZ = 1024, 2.4
# VALU ceiling for this exact instruction mix: a wave64 half-rate op holds the
# SIMD 4 clocks, a full-rate op 2 -> 1994 clocks per 64-byte block per wave.
_MIX_CLK = 4 * VALU_HALF_RATE_PER_BLOCK + 2 * VALU_FULL_RATE_PER_BLOCK
VALU_MIX_PEAK_TOPS = VALU_OPS_PER_BLOCK * 64 * SIMDS * CLOCK_GHZ * 1e9 / _MIX_CLK / 1e12  # lane-ops/s, ~47.1
METRIC = "GiB/s SHA-1 hashed (device-resident 512KiB chunks) at 1/2/4/8 MI355X"
DEFAULT_VARIANT = (3, 1, 0)  # the product library's one hot kernel


def process_age_s():
    """Seconds since THIS process started (kernel start time from
    /proc/self/stat against /proc/uptime, 1/CLK_TCK resolution), i.e. from
    interpreter start -- what the driver's clock around `python bench.py` sees,
    minus the exec.  Falls back to the time since bench.py was imported."""
    try:
        with open("/proc/self/stat") as f:
            after_comm = f.read().rsplit(")", 1)[1].split()
        start_ticks = int(after_comm[19])  # field 22 of stat(5); field 3 is after_comm[0]
        with open("/proc/uptime") as f:
            uptime = float(f.read().split()[0])
        return round(uptime - start_ticks / os.sysconf("SC_CLK_TCK"), 2)
    except (OSError, ValueError, IndexError):
        return round(time.perf_counter() - _T_IMPORT, 2)


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


EXPERIMENTS_LIB = os.path.join(HERE, "build_variants", "experiments", "libbtsha1.so")


def ensure_built(experiments=False):
    """A clean checkout has no built artefacts (git-ignored): build the library,
    its host tools and the test-only oracle once (N ranks start together) --
    and, for a non-default --ring/--lines/--nt variant, the experiments library
    that alone carries the rejected hot-kernel variants."""
    need = [os.path.join(PKG, "libbtsha1.so"), os.path.join(PKG, "bin", "verify-stream"),
            os.path.join(HERE, "oracle", "liboracle_sha1.so"), os.path.join(HERE, "oracle", "liboracle_sha1_O0.so")]
    targets = ["lib", "tools", "oracle"]
    if experiments:
        need.append(EXPERIMENTS_LIB)
        targets.append("experiments")
    if all(os.path.exists(p) for p in need):
        return
    import fcntl
    with open(os.path.join(HERE, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not all(os.path.exists(p) for p in need):
            subprocess.run(["make", "-C", HERE, "-j8", *targets], check=True)


# ---------------------------------------------------------------------------
# --gpus N is authoritative (the driver's `python bench.py --gpus N` and its
# torchrun launch both end up as N ranks, or the run fails before any GPU call)
# ---------------------------------------------------------------------------
def rank_plan(gpus, environ):
    """("single" | "spawn" | "ranks", error message or None) for `--gpus
    gpus` under `environ` -- decided before torch is imported:
      * WORLD_SIZE unset, gpus == 1: this process is the one rank;
      * WORLD_SIZE unset, gpus > 1: start the N ranks as a torch.distributed.run
        child (spawn_ranks) and relay rank 0's line;
      * WORLD_SIZE set: a launcher started us as one of its ranks, and its
        world size must be exactly --gpus (a mismatch is a launch error: the
        line would claim a GPU count it did not run on)."""
    if gpus < 1:
        return None, f"--gpus {gpus}: need at least one GPU"
    ws = environ.get("WORLD_SIZE")
    if ws is None or ws == "":
        return ("single" if gpus == 1 else "spawn"), None
    try:
        world = int(ws)
    except ValueError:
        return None, f"WORLD_SIZE={ws!r} is not an integer"
    if world != gpus:
        return None, (f"launched as one of WORLD_SIZE={world} ranks but --gpus {gpus}: the launcher's world size and "
                      f"--gpus must agree (run `python bench.py --gpus {gpus}` alone, or launch {gpus} ranks)")
    return "ranks", None


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(n, argv, port):
    """The driver's own N > 1 launch line (one process per GPU, 127.0.0.1
    rendezvous), running this file with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def relay(cmd, env=None):
    """Run `cmd` as a child process (never exec: nothing here has touched the
    GPU, but the ranks will) and relay its result line: the child's JSON
    line(s) are held back and exactly one is printed on our stdout; every
    other stdout line goes to stderr as it arrives, stderr passes straight
    through (progress stays visible).  SIGTERM is forwarded to the child, and
    the child gets SIGTERM if this process dies (PR_SET_PDEATHSIG), so the
    ranks never outlive their parent.  Returns the child's exit status, or 1
    when it exited 0 without exactly one JSON line."""
    def die_with_parent():
        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGTERM))  # PR_SET_PDEATHSIG

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1, preexec_fn=die_with_parent)
    prev = signal.signal(signal.SIGTERM, lambda sig, _frame: p.send_signal(sig))
    lines = []
    try:
        for text in p.stdout:
            if text.startswith("{"):
                lines.append(text.rstrip("\n"))
            else:
                sys.stderr.write(text)
                sys.stderr.flush()
        rc = p.wait()
    finally:
        signal.signal(signal.SIGTERM, prev)
    if len(lines) == 1:
        print(lines[0], flush=True)
    elif rc == 0:
        print(f"bench.py: the rank launch printed {len(lines)} result lines, expected exactly 1", file=sys.stderr,
              flush=True)
        return 1
    return exit_status(rc)


def exit_status(rc):
    """A child's returncode as this process's exit status: a child killed by
    signal S (returncode -S) becomes the shell's 128 + S, not sys.exit(-S)'s
    256 - S, so the driver sees a signal death as one."""
    return 128 - rc if rc < 0 else rc


def spawn_ranks(n, argv):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool
    cmd = rank_launch_cmd(n, argv, free_port())
    print(f"bench.py: --gpus {n} without a launcher: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    return relay(cmd, env)


# ---------------------------------------------------------------------------
# The HIP hasher one rank drives (shard.run_rank protocol).
# ---------------------------------------------------------------------------
class DeviceHasher:
    def __init__(self, bt, torch, chunks, pitch, first_chunk):
        self.bt, self.torch, self.C, self.pitch = bt, torch, chunks, pitch
        self.buf = torch.empty(pitch * (chunks - 1) + CHUNK + 256, dtype=torch.uint8, device="cuda")
        self.dig = torch.zeros(20 * chunks, dtype=torch.uint8, device="cuda")
        # A dedicated stream: kernels and timing events share it.
        self.stream = torch.cuda.Stream()
        self.sp = self.stream.cuda_stream
        if pitch == CHUNK:
            bt.fill_synthetic(self.buf.data_ptr(), chunks * CHUNK, first_chunk * (CHUNK // 8), SEED, self.sp)
        else:  # padded layout: fill chunk by chunk (same bytes per chunk)
            for i in range(chunks):
                bt.fill_synthetic(self.buf.data_ptr() + i * pitch, CHUNK, (first_chunk + i) * (CHUNK // 8), SEED, self.sp)
        torch.cuda.synchronize()
        self.ev = []

    def step(self, i):
        if i >= 0:
            a, b = self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True)
            a.record(self.stream)
            self.bt.chunks_dev(self.buf.data_ptr(), self.C, CHUNK, self.pitch, self.dig.data_ptr(), self.sp)
            b.record(self.stream)
            self.ev.append((a, b))
        else:
            self.bt.chunks_dev(self.buf.data_ptr(), self.C, CHUNK, self.pitch, self.dig.data_ptr(), self.sp)

    def sync(self):
        self.torch.cuda.synchronize()

    def kernel_ms(self):
        return sum(a.elapsed_time(b) for a, b in self.ev) / len(self.ev) if self.ev else None

    def kernel_ms_median(self):
        """SURVEY.md §8d's config-3 statistic (median of the timed launches)."""
        if not self.ev:
            return None
        t = sorted(a.elapsed_time(b) for a, b in self.ev)
        return (t[(len(t) - 1) // 2] + t[len(t) // 2]) / 2

    def digests(self):
        return self.dig.cpu().numpy().tobytes()

    def verify_rate(self, pairs=6):
        """Device-resident verify (util.c:311-313's hash + memcmp, batched):
        bt_sha1_verify_dev over the same chunks against expected digests in
        HBM, every 997th deliberately wrong, measured PAIRED with the plain
        hash it extends: `pairs` pairs of one chunks_dev and one verify_dev
        launch, interleaved on the hasher's stream in one window in ABBA order
        (hash-verify, verify-hash, ...) so clock / power drift falls on both
        kernels alike, each launch timed with its own HIP events.  One untimed
        launch of each first (the first launch of the verify instantiation
        pays a one-time cost, ~3 ms in rocprof traces).  Reports both means,
        the overhead of the fused compare and its spread over the pairs, and
        whether exactly the wrong chunks were flagged."""
        import statistics
        torch = self.torch
        ev = torch.cuda.Event
        with torch.cuda.stream(self.stream):
            exp = self.dig.clone()
            bad = torch.arange(0, self.C, 997, device="cuda")
            exp.view(-1, 20)[bad, 0] ^= 1
            ok = torch.full((self.C,), 7, dtype=torch.uint8, device="cuda")

            def launch(kind):
                if kind == "verify":
                    self.bt.verify_dev(self.buf.data_ptr(), self.C, CHUNK, self.pitch, exp.data_ptr(),
                                       ok.data_ptr(), None, self.sp)
                else:
                    self.bt.chunks_dev(self.buf.data_ptr(), self.C, CHUNK, self.pitch, self.dig.data_ptr(), self.sp)
            launch("verify")
            launch("hash")
            ok.fill_(7)  # the timed passes must set every flag themselves
            timed = []
            for p in range(pairs):
                for kind in (("hash", "verify") if p % 2 == 0 else ("verify", "hash")):
                    a, b = ev(enable_timing=True), ev(enable_timing=True)
                    a.record(self.stream)
                    launch(kind)
                    b.record(self.stream)
                    timed.append((p, kind, a, b))
        torch.cuda.synchronize()
        ms = {(p, k): a.elapsed_time(b) for p, k, a, b in timed}
        hash_ms = [ms[(p, "hash")] for p in range(pairs)]
        ver_ms = [ms[(p, "verify")] for p in range(pairs)]
        per_pair = [100.0 * (v / h - 1.0) for h, v in zip(hash_ms, ver_ms)]
        h_mean, v_mean = statistics.mean(hash_ms), statistics.mean(ver_ms)
        want = torch.ones(self.C, dtype=torch.uint8, device="cuda")
        want[bad] = 0
        return {"GiB_per_s": round(self.C * CHUNK / (v_mean * 1e-3) / 2**30, 3), "kernel_ms": round(v_mean, 4),
                "hash_ms": round(h_mean, 4), "verify_ms": round(v_mean, 4),
                "overhead_pct": round(100.0 * (v_mean / h_mean - 1.0), 3),
                "overhead_pct_pairs": {"min": round(min(per_pair), 3), "median": round(statistics.median(per_pair), 3),
                                       "max": round(max(per_pair), 3)},
                "pairs": pairs,
                "flags_correct": bool(torch.equal(ok, want)), "mismatches_planted": int(bad.numel()),
                "kernel": self.bt.kernel_name(self.C),
                "path": "bt_sha1_verify_dev (fused compare, util.c:311-313) vs bt_sha1_chunks_dev: ABBA pairs "
                        "in one window, per-launch HIP events, one untimed launch of each first"}

    def clock_mhz(self, launches=3):
        """Median in-kernel shader clock over the waves of the last of
        `launches` back-to-back launches of the stamped build, right after the
        timed region (MI355X_MICROARCH.md, DVFS item 6)."""
        torch = self.torch
        waves = (self.C + 63) // 64
        # zero-filled on the hasher's own stream, so the fills are ordered
        # before the probe's stamp / digest writes
        with torch.cuda.stream(self.stream):
            st = torch.zeros(4 * waves, dtype=torch.int64, device="cuda")
            scratch = torch.zeros(20 * self.C, dtype=torch.uint8, device="cuda")
        for _ in range(launches):
            self.bt.clock_probe(self.buf.data_ptr(), self.C, CHUNK, self.pitch, scratch.data_ptr(), st.data_ptr(), self.sp)
        torch.cuda.synchronize()
        s = st.view(-1, 4).cpu().double()
        ratio = ((s[:, 2] - s[:, 0]) / (s[:, 3] - s[:, 1])).median().item()
        same = bool(torch.equal(scratch, self.dig))
        return ratio * self.bt.wallclock_khz() / 1000.0, same


# ---------------------------------------------------------------------------
# Board power while the hot kernel runs (the kernel is bounded by
# the board power limit, not by HBM or VALU issue)
# ---------------------------------------------------------------------------
def _smi_matches(torch, dev):
    """(amdsmi module, every processor handle at HIP device `dev`'s PCI
    domain:bus:device) -- a box may expose one GPU to HIP and several to
    amdsmi; partitions of one GPU share domain:bus:device and differ only in
    the function number, which HIP does not report."""
    import amdsmi
    amdsmi.amdsmi_init()
    p = torch.cuda.get_device_properties(dev)
    want = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    hits = []
    for h in amdsmi.amdsmi_get_processor_handles():
        dom, bus, rest = amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")
        if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
            hits.append(h)
    return amdsmi, hits


def _smi_handle(torch, dev):
    """(amdsmi module, the first processor handle at HIP device `dev`'s PCI
    address, or None) -- for the power reading (partitions share a socket)."""
    smi, hits = _smi_matches(torch, dev)
    return smi, (hits[0] if hits else None)


def device_identity(torch, dev):
    """Which physical GPU this rank drives: its host; its PCI address as HIP
    reports it (`pci_bdf`, domain:bus:device with the function number fixed
    at .0 -- HIP does not expose it) and as amdsmi reports it (`smi_bdf`,
    with the real function number); the UUID amdsmi holds for that address
    (`uuid_source` "smi"), or the `uuid` HIP exposes through torch when
    amdsmi fails ("hip", written differently for the same GPU); the HIP
    device index and how many devices the rank can see -- so an N > 1 line
    proves it ran on N distinct GPUs (shard.check_distinct_devices)."""
    p = torch.cuda.get_device_properties(dev)
    ident = {"pci_bdf": f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}.0",
             "uuid": None, "uuid_source": None, "hip_device": dev, "device_count": torch.cuda.device_count(),
             "name": p.name, "host": socket.gethostname()}
    smi = None
    try:
        smi, hits = _smi_matches(torch, dev)
        if len(hits) == 1:
            h = hits[0]
            ident["uuid"] = str(smi.amdsmi_get_gpu_device_uuid(h))
            ident["uuid_source"] = "smi"
            ident["smi_bdf"] = str(smi.amdsmi_get_gpu_device_bdf(h))
        elif hits:  # which partition this HIP device is cannot be told apart: HIP's fields only
            ident["smi_error"] = f"{len(hits)} amdsmi devices at this PCI address (partitions of one GPU)"
    except Exception as e:  # noqa: BLE001 -- identity falls back to HIP's own fields
        ident["smi_error"] = f"{type(e).__name__}: {e}"
    finally:
        if smi is not None:
            try:
                smi.amdsmi_shut_down()
            except Exception:  # noqa: BLE001
                pass
    if ident["uuid"] is None and getattr(p, "uuid", None) is not None:
        ident["uuid"] = str(p.uuid)
        ident["uuid_source"] = "hip"
    return ident


def power_window(hasher, torch, dev, seconds):
    """Run the timed step back to back for ~`seconds` after the timed region
    and report the socket power from the SMU energy accumulator (delta energy /
    delta wall time) and from current_socket_power samples (every 50 ms), with
    the power cap, the per-XCD gfx clocks and the energy per GiB hashed."""
    smi, h = _smi_handle(torch, dev)
    try:
        if h is None:
            return {"error": "no amdsmi device with this GPU's PCI address"}
        return _power_window(smi, h, hasher, seconds)
    finally:
        smi.amdsmi_shut_down()


def _power_window(smi, h, hasher, seconds):
    import statistics
    limit_w = smi.amdsmi_get_power_cap_info(h)["power_cap"] / 1e6  # reported in microwatts
    per_launch_ms = hasher.kernel_ms() or 20.0
    n = max(2, int(seconds * 1e3 / per_launch_ms))
    samples, stop = [], threading.Event()

    def sampler():
        while not stop.is_set():
            try:
                m = smi.amdsmi_get_gpu_metrics_info(h)
                clks = [c for c in m.get("current_gfxclks", []) if isinstance(c, (int, float))]
                samples.append((float(m["current_socket_power"]), statistics.median(clks) if clks else None))
            except Exception:  # noqa: BLE001 -- a missed sample is not an error
                pass
            stop.wait(0.05)

    hasher.sync()
    m0 = smi.amdsmi_get_gpu_metrics_info(h)
    e0, t0 = smi.amdsmi_get_energy_count(h), time.perf_counter()
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    for _ in range(n):
        hasher.step(-1)
    hasher.sync()
    t1, e1 = time.perf_counter(), smi.amdsmi_get_energy_count(h)
    m1 = smi.amdsmi_get_gpu_metrics_info(h)
    stop.set()
    th.join()
    # Which limiter held the clock: the SMU's residency accumulators count the
    # ticks (of accumulation_counter) each one was active over the window.
    ticks = m1.get("accumulation_counter", 0) - m0.get("accumulation_counter", 0)
    residency = {k[:-len("_residency_acc")]: round((m1[k] - m0[k]) / ticks, 4) for k in sorted(m1)
                 if k.endswith("_residency_acc") and isinstance(m1[k], int) and isinstance(m0.get(k), int)
                 and ticks > 0}
    joules = (e1["energy_accumulator"] - e0["energy_accumulator"]) * e0["counter_resolution"] * 1e-6
    watts = joules / (t1 - t0)
    gibps = n * hasher.C * CHUNK / (t1 - t0) / 2**30
    # the second half of the samples: after the power controller has settled
    steady = samples[len(samples) // 2:]
    sw = [w for w, _ in steady]
    sc = [c for _, c in steady if c]
    return {
        "socket_W": round(watts, 1), "power_cap_W": round(limit_w, 1), "frac_of_cap": round(watts / limit_w, 4),
        "sampled_socket_W_median": round(statistics.median(sw), 1) if sw else None,
        "gfxclk_MHz_median": round(statistics.median(sc), 1) if sc else None,
        "J_per_GiB": round(watts / gibps, 3), "GiB_per_s": round(gibps, 3),
        "limiter_residency": residency,
        "temperature_C": {k: m1.get(f"temperature_{k}") for k in ("hotspot", "mem")},
        "launches": n, "window_s": round(t1 - t0, 3), "samples": len(samples),
        "method": "timed step back to back after the timed region; socket_W = SMU energy accumulator delta / "
                  "wall; samples every 50 ms (median of the 2nd half); limiter_residency = fraction of SMU ticks",
    }


# ---------------------------------------------------------------------------
# CPU baseline
# ---------------------------------------------------------------------------
def usable_cores():
    """(threads this process may run on, machine CPUs, cgroup quota in CPUs or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, math.ceil(quota)))
    return threads, os.cpu_count(), quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(host_addr, n_chunks, gpu_digests, min_s=1.0, reps=3):
    """Reference sha.c (or our port when the reference objects are absent)
    hashing n_chunks 512 KiB chunks at host_addr, shahash per chunk as
    chunk.c:21 does, at 1 thread, at the CPUs the cgroup quota pays for and
    (-O2) at one thread per CPU of the affinity mask; -O2 and the reference
    Makefile's -O0.

    Sustained, not burst: every measurement repeats passes over the sample
    until it has run >= min_s (>= 10 CFS periods, so a quota'd cgroup cannot
    ride on burst credit) and the rate is the median of `reps` measurements.
    1-thread legs use the first quarter of the sample (>= 256 chunks) so the
    leg stays ~1 s per measurement.  `cores` is the CPU budget actually usable,
    min(affinity, ceil(quota)); the thread count of each run is reported
    separately."""
    import statistics
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import py_oracle  # test infrastructure: the checker / baseline, never the product
    out = (ctypes.c_uint8 * (20 * n_chunks))()
    cores, machine, quota = usable_cores()
    affinity = len(os.sched_getaffinity(0))

    def pick(opt):
        ref = py_oracle.load_reference(opt)
        if ref is not None:
            return "reference", ref.shahash
        port = py_oracle.load_port(opt)
        return ("port", port.or_shahash) if port is not None else (None, None)

    def one_pass(fn, nthreads, n):
        def hash_range(lo, hi):
            for i in range(lo, hi):  # ctypes drops the GIL inside each call
                fn(ctypes.c_void_p(host_addr + i * CHUNK), CHUNK, ctypes.byref(out, 20 * i))
        ts = [threading.Thread(target=hash_range, args=(n * t // nthreads, n * (t + 1) // nthreads))
              for t in range(nthreads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    def run(fn, nthreads, n):
        rates, passes = [], 0
        # each leg's parity flag must reflect its own writes, not an earlier leg's
        ctypes.memset(out, 0, ctypes.sizeof(out))
        for _ in range(reps):
            t0, k = time.perf_counter(), 0
            while True:
                one_pass(fn, nthreads, n)
                k += 1
                dt = time.perf_counter() - t0
                if dt >= min_s:
                    break
            rates.append(k * n * CHUNK / dt / 2**30)
            passes += k
        ok = bytes(out)[:20 * n] == gpu_digests[:20 * n]
        return {"GiB_per_s": round(statistics.median(rates), 4),
                "spread": round((max(rates) - min(rates)) / statistics.median(rates), 4),
                "sample_chunks": n, "passes": passes, "digests_match_gpu": ok}

    n1 = max(min(256, n_chunks), n_chunks // 4)
    rows, kind, run_flags = {}, None, {}
    for opt, flags in (("O2", "-O2"), ("O0", "-g -O0 (reference Makefile:3)")):
        k, fn = pick(opt)
        if fn is None:
            continue
        kind = kind or k
        run_flags[opt] = flags
        counts = {1, cores} | ({affinity} if opt == "O2" else set())
        for nt in sorted(counts):
            r = run(fn, nt, n1 if nt == 1 else n_chunks)
            # a run's flags are its key's prefix (run_flags); its kind only when it differs
            rows[f"{opt}_{nt}t"] = {**r, "threads": nt, **({"kind": k} if k != kind else {})}
    # value: the best sustained -O2 rate over the multi-thread runs (`cores`
    # threads, one per CPU of the affinity mask); both are bounded by the
    # quota, and with exactly `cores` threads the process's other threads
    # (interpreter, HIP runtime) make that run the noisier of the two.
    multi = [r for key, r in rows.items() if key.startswith("O2_") and r["threads"] > 1]
    head = max(multi, key=lambda r: r["GiB_per_s"]) if multi else (rows.get("O2_1t") or next(iter(rows.values())))
    per_core = rows.get("O2_1t", {}).get("GiB_per_s")
    return {
        "value": head["GiB_per_s"], "unit": "GiB/s", "cores": cores, "threads": head["threads"], "kind": kind,
        "sample": f"{n_chunks} x 512 KiB of the bench's chunks ({n1} on 1 thread), shahash per chunk (chunk.c:21); "
                  f"rate = median of {reps} runs of >= {min_s:g} s; value = best -O2 multi-thread run; cores = "
                  f"min(affinity {affinity}, ceil(quota {quota}))",
        "flags": run_flags.get("O2"), "digests_match_gpu": all(r["digests_match_gpu"] for r in rows.values()),
        "per_core_GiB_per_s_O2": per_core,
        "quota_bound_GiB_per_s": round(per_core * quota, 3) if per_core and quota else None,
        "runs": rows, "run_flags": run_flags, "machine_cpus": machine, "affinity_cpus": affinity,
        "cgroup_cpu_quota": quota, "host_cpu": cpu_model(),
    }


# ---------------------------------------------------------------------------
# Host paths (config 5): PCIe-inclusive, starting in host memory
# ---------------------------------------------------------------------------
def cgroup_cpu_stat():
    """This process's cgroup CPU accounting (cgroup v2 cpu.stat): usage and
    time throttled by the CPU quota, in seconds; None where unreadable."""
    try:
        d = dict(l.split() for l in open("/sys/fs/cgroup/cpu.stat") if l.strip())
        return {"usage_s": int(d["usage_usec"]) / 1e6, "throttled_s": int(d.get("throttled_usec", 0)) / 1e6,
                "nr_throttled": int(d.get("nr_throttled", 0))}
    except (OSError, ValueError, KeyError):
        return None


def machine_cpu_ticks():
    """(busy, total) jiffies of the whole machine (/proc/stat `cpu` line: not
    namespaced, so it counts every tenant of the host, not only this job)."""
    try:
        with open("/proc/stat") as f:
            v = [int(x) for x in f.readline().split()[1:]]
        idle = v[3] + (v[4] if len(v) > 4 else 0)
        return sum(v) - idle, sum(v)
    except (OSError, ValueError, IndexError):
        return None


def timed_runs(fn, want, gib, steady=5, stats=None):
    """The first run of a host path (it also pays one-time pinning / page
    locking), then `steady` more; value = the MEDIAN steady run.  Every run's
    rate is listed; the median run and the first run carry their breakdown
    (HOST_PATH_FIELDS): wall time, this process's CPU time, the time the
    cgroup's quota throttled it, the whole machine's CPU busy fraction and --
    with stats (bt.pipeline_stats) -- the pipeline's own phase split."""
    import statistics
    runs, ok = [], True
    for _ in range(1 + steady):
        cg0, cpu0, m0 = cgroup_cpu_stat(), time.process_time(), machine_cpu_ticks()
        t0 = time.perf_counter()
        r = fn()
        dt = time.perf_counter() - t0
        cpu, cg1, m1 = time.process_time() - cpu0, cgroup_cpu_stat(), machine_cpu_ticks()
        ok = ok and r == want
        row = {"GiB_per_s": round(gib / dt, 3), "s": round(dt, 4), "cpu_s": round(cpu, 3)}
        if cg0 and cg1:
            row["throttled_s"] = round(cg1["throttled_s"] - cg0["throttled_s"], 4)
        if m0 and m1 and m1[1] > m0[1]:
            row["host_busy"] = round((m1[0] - m0[0]) / (m1[1] - m0[1]), 3)
        if stats is not None:
            st = stats()
            row.update(fill_s=st["fill_s"], wait_s=st["wait_s"], alloc_s=st["alloc_s"], lock_s=st["register_s"],
                       unlock_s=st["unregister_s"])
        runs.append(row)
    steady_rates = [r["GiB_per_s"] for r in runs[1:]]
    mid = sorted(runs[1:], key=lambda r: r["GiB_per_s"])[len(runs[1:]) // 2]
    out = {"GiB_per_s": round(statistics.median(steady_rates), 3), "first_run_GiB_per_s": runs[0]["GiB_per_s"],
           "runs_GiB_per_s": [r["GiB_per_s"] for r in runs], "digests_match": ok,
           "median_run": {k: v for k, v in mid.items() if k != "GiB_per_s"},
           "first_run": {k: v for k, v in runs[0].items() if k in ("s", "alloc_s", "lock_s", "fill_s", "wait_s")}}
    if stats is not None and mid["s"] > 0:
        out["median_run"]["fill_frac"] = round(mid["fill_s"] / mid["s"], 3)
    return out


HOST_PATH_FIELDS = (
    "GiB_per_s: median of runs 2-6; median_run/first_run: s wall, cpu_s, throttled_s (cgroup), host_busy (whole "
    "machine), fill_s (host input copies), wait_s (on the GPU lane), lock_s/unlock_s (page locking); numa: feed, "
    "locked/all batches, column-split tail chunks, GPU node, image/lane pages and staging pieces per node")


def numa_view(st):
    """How a pipeline run was fed and where its memory sat, from
    bt_sha1_get_pipeline_stats (fields in HOST_PATH_FIELDS)."""
    return {"feed": st["feed"], "locked_batches": [st["registered_batches"], st["batches"]],
            "column_chunks": st["column_chunks"],
            "gpu_node": st["gpu_numa_node"], "image_pages": st["src_pages"], "lane_pages": st["lane_pages"],
            "staging_pieces": st["copy_pieces"], "policy": st["numa_policy"], "copy_threads": st["copy_threads"]}


def run_verify_stream(vs, args, timeout=300):
    """One bin/verify-stream run; its JSON summary beside the digests check."""
    r = subprocess.run([vs, *args], capture_output=True, text=True, timeout=timeout)
    lines = r.stdout.strip().splitlines()
    try:
        res = json.loads(lines[-1]) if lines else {}
    except ValueError:
        res = {}
    row = {"GiB_per_s": res.get("GiB_per_s"),
           "digests_match": r.returncode == 0 and res.get("failed") == 0 and res.get("ok") == res.get("chunks"),
           "chunks": res.get("chunks"), "timed_chunks": res.get("timed_chunks"),
           "receive_threads": res.get("receive_threads"), "args": " ".join(args[:-2])}
    if res.get("late_fills"):
        row["late_fills"] = res["late_fills"]
    if r.returncode != 0:
        row["error"] = f"rc={r.returncode} {r.stderr[-300:]} {lines[-1:]}"
    return row


def host_paths(bt, torch, dev_buf, host, want, verify_gib=1):  # noqa: C901
    """host: pageable numpy image of the first chunks of dev_buf; want: their
    device-resident digests.  Each pipeline rate is the median of 5
    steady-state runs after a first one (which also pays one-time pinning /
    page locking); the fields are described in the line itself (`fields`)."""
    addr, nbytes = host.ctypes.data, host.nbytes
    gib = nbytes / 2**30
    out = {"image_GiB": round(gib, 3), "fields": HOST_PATH_FIELDS}

    # Pageable image, default feed: each ~1 GiB batch's whole pages page-locked
    # (all before the first copy, released after the last batch), DMA'd in
    # place, unaligned edge bytes through a pinned buffer.
    out["pageable_chunks_host"] = {
        **timed_runs(lambda: bt.chunks_host_addr(addr, nbytes), want, gib, stats=bt.pipeline_stats),
        "numa": numa_view(bt.pipeline_stats())}
    # The same call with the staged feed: 8 threads copy every byte into
    # page-locked lanes (on the GPU's NUMA node) ahead of the H2D -- its rate
    # follows the host's spare memory bandwidth and cores.
    prev = bt.set_pageable_feed("stage")
    try:
        out["pageable_staged_copy"] = {
            **timed_runs(lambda: bt.chunks_host_addr(addr, nbytes), want, gib, stats=bt.pipeline_stats),
            "numa": numa_view(bt.pipeline_stats())}
    finally:
        bt.set_pageable_feed(prev)
    t0 = time.perf_counter()
    bt.host_register(addr, nbytes)
    reg_s = time.perf_counter() - t0
    try:
        # the caller registered the whole image: DMA straight from it
        out["registered_direct_dma"] = {
            **timed_runs(lambda: bt.chunks_host_addr(addr, nbytes), want, gib, stats=bt.pipeline_stats),
            "register_s": round(reg_s, 3)}
        del out["registered_direct_dma"]["first_run"]  # nothing one-time left: the caller registered the image
        pin = torch.from_numpy(host)
        scratch = torch.empty(nbytes, dtype=torch.uint8, device=dev_buf.device)
        rates = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            scratch.copy_(pin, non_blocking=True)
            torch.cuda.synchronize()
            rates.append(round(gib / (time.perf_counter() - t0), 3))
        del scratch
        out["raw_h2d_ceiling"] = {"GiB_per_s": max(rates), "runs": rates}  # one hipMemcpy of the registered image
    finally:
        bt.host_unregister(addr)
    for key in ("pageable_chunks_host", "pageable_staged_copy", "registered_direct_dma"):
        out[key]["frac_of_raw_h2d"] = round(out[key]["GiB_per_s"] / out["raw_h2d_ceiling"]["GiB_per_s"], 4)
    # The batched verifier (util.c:304-337 replacement): the product's C host
    # tool over a 1 GiB image in a tmpfs file.  Zero-copy: the receive landed
    # the bytes in the pinned slots once, the 8 timed rounds re-verify them
    # (the H2D + hash + verdict bound).  Packetized: every timed round receives
    # each chunk again as util.c:275 does -- 1484-byte memcpys into the slot --
    # on one receive thread, and on four (four verifiers, -g 4 -t); 2 rounds
    # timed after 1 untimed.
    vs = os.path.join(PKG, "bin", "verify-stream")
    n = min(int(verify_gib * 2**30) // CHUNK, nbytes // CHUNK)
    import shutil
    shm = "/dev/shm"
    if not os.path.isdir(shm) or shutil.disk_usage(shm).free < 2 * n * CHUNK:
        shm = tempfile.gettempdir()
    with tempfile.TemporaryDirectory(dir=shm) as d:
        img, lst = os.path.join(d, "img"), os.path.join(d, "img.chunks")
        host[:n * CHUNK].tofile(img)
        with open(lst, "w") as f:
            for i in range(n):
                f.write(f"{i} {want[20 * i:20 * i + 20].hex()}\n")
        out["zero_copy_verifier"] = run_verify_stream(vs, ["-z", "-b", "1024", "-s", "2", "-r", "9", img, lst])
        out["packetized_verifier"] = run_verify_stream(vs, ["-b", "1024", "-s", "2", "-r", "3", "-w", "1", img, lst])
        out["packetized_verifier_4_threads"] = run_verify_stream(
            vs, ["-g", "4", "-t", "-b", "256", "-s", "2", "-r", "3", "-w", "1", img, lst])
    return out


def find_traffic(want, path=None):
    """(HBM bytes per launch, note) from the PMC traffic file measured on this
    very build -- source id, kernel, variant and layout all equal to `want` --
    else (None, why).  Default: the newest profiles/traffic_r*.json that
    matches."""
    paths = [path] if path else sorted(glob.glob(os.path.join(HERE, "profiles", "traffic_r*.json")), reverse=True)
    tried = []
    for p in paths:
        rel = os.path.relpath(p, HERE)
        try:
            tj = json.load(open(p))
        except (OSError, ValueError) as e:
            tried.append(f"{rel}: unreadable ({e})")
            continue
        diff = {k: (tj.get(k), v) for k, v in want.items() if tj.get(k) != v}
        if not diff:
            return tj.get("hbm_bytes_per_launch"), f"{rel} (rocprofv3 --pmc, same source id)"
        tried.append(f"{rel} was measured on another build/layout: {diff}")
    return None, "; ".join(tried) or "no PMC traffic file for this build"


# ---------------------------------------------------------------------------
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
    ap.add_argument("--cpu-chunks", type=int, default=4096, help="CPU-baseline sample (SURVEY.md §8d: 4096 chunks)")
    ap.add_argument("--host-gib", type=float, default=8.0, help="host-path image size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-clock", action="store_true")
    ap.add_argument("--power-s", type=float, default=2.0,
                    help="seconds of back-to-back steps after the timed region for the board-power reading (0 = off)")
    ap.add_argument("--backend", default="gloo",
                    help="process group for the control plane (barriers, timings, digest gather); "
                         "the hash path has no collective")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic file (default: the newest profiles/traffic_r*.json measured on this "
                         "build's source id, kernel, variant and layout)")
    ap.add_argument("--digest-sample", type=int, default=3,
                    help="digests of this many chunks of EVERY rank (first, last, evenly between) in the line, "
                         "for parity checks beyond the golden range (0 = off)")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="allow N > 1 ranks on fewer than N distinct GPUs (a rehearsal of the rank path on one "
                         "GPU, recorded in the line); without it such a launch exits before the timed region")
    args = ap.parse_args()

    if args.steps < 1 or args.warmup < 0 or args.chunks < 1:
        print(f"bench.py: need --steps >= 1, --warmup >= 0 and --chunks >= 1 (got {args.steps}, {args.warmup}, "
              f"{args.chunks})", file=sys.stderr, flush=True)
        sys.exit(2)
    # Before torch is imported or any GPU call: --gpus decides the rank count.
    plan, err = rank_plan(args.gpus, os.environ)
    if err:
        print(f"bench.py: {err}", file=sys.stderr, flush=True)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    phases = {}
    t_phase = time.perf_counter()

    def phase(name):
        nonlocal t_phase
        now = time.perf_counter()
        phases[name] = round(now - t_phase, 2)
        t_phase = now

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())  # == local on a full node
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            group = dist.new_group(backend="gloo")
        else:
            dist.init_process_group(args.backend)
    variant = (args.ring, args.lines, args.nt) if args.ring else DEFAULT_VARIANT
    experiments = variant != DEFAULT_VARIANT and "BT_SHA1_LIB" not in os.environ
    if rank == 0:
        ensure_built(experiments)
    shard.barrier(world, group)
    if experiments:
        # the rejected hot-kernel variants exist only in the experiments build
        os.environ["BT_SHA1_LIB"] = EXPERIMENTS_LIB
    bt = _load("btsha1", os.path.join(PKG, "btsha1.py"))
    if args.ring:
        bt.set_variant(*variant)

    C, pitch = args.chunks, args.pitch
    first_chunk, last_chunk = shard.weak_range(rank, C)
    kernel = bt.kernel_name(C)
    # Which GPU each rank drives, before anything is allocated or timed: an
    # N > 1 line must show N distinct devices (PCI address + UUID per rank).
    ident = dict(rank=rank, **device_identity(torch, dev), kernel=kernel, chunk_range=[first_chunk, last_chunk])
    idents = shard.gather_objects(ident, world, group)
    clash = shard.check_distinct_devices(idents, world, allow_shared=args.rehearse_shared_gpu)
    if clash:
        print(f"bench.py rank {rank}: {clash}", file=sys.stderr, flush=True)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(3)
    phase("init_s")
    hasher = DeviceHasher(bt, torch, C, pitch, first_chunk)
    phase("fill_s")
    res = shard.run_rank(hasher, args.steps, args.warmup, world, rank, group)
    phase("warmup_and_timed_s")

    # Every rank stamps its own GPU's in-kernel clock (all ranks together,
    # after the timed region), so a slow rank of an N-GPU line is attributable
    # to its clock or to its kernel without a second run.
    clock, rank_mhz = None, None
    if not args.no_clock and kernel == "k_sha1_fixed":
        mine, err = [-1.0, 0.0], None
        try:
            mhz, same = hasher.clock_mhz()
            mine = [mhz, 1.0 if same else 0.0]
        except Exception as e:  # noqa: BLE001 -- the clock evidence must never cost the bench line
            err = f"{type(e).__name__}: {e}"
        allc = shard.gather_floats(mine, world, group)
        rank_mhz = [round(m, 1) if m > 0 else None for m, _ in allc]
        ok = [m for m in rank_mhz if m is not None]
        if ok:
            slow = min(range(world), key=lambda r: rank_mhz[r] if rank_mhz[r] is not None else math.inf)
            clock = {"in_kernel_mhz": min(ok), "probe_digests_identical": all(s > 0 for _, s in allc),
                     "method": "stamped hot kernel (bt_sha1_clock_probe): median over waves of d(s_memtime) / "
                               "d(s_memrealtime) x wall-clock rate, 3 launches after the timed region, every rank"}
            if world > 1:
                clock.update(slowest_rank=slow, per_rank_mhz=rank_mhz,
                             note="in_kernel_mhz = the slowest rank's clock (it prices the VALU roofline)")
            if len(ok) < world:
                clock["missing_ranks"] = [r for r in range(world) if rank_mhz[r] is None]
        else:
            clock = {"error": err or "no rank reported a clock"}
        phase("clock_s")

    # Every rank measures its own GPU's power (all ranks run the window together).
    power = None
    if args.power_s > 0:
        try:
            power = power_window(hasher, torch, dev, args.power_s)
        except Exception as e:  # noqa: BLE001 -- the power evidence must never cost the bench line
            power = {"error": f"{type(e).__name__}: {e}"}
        keys = ("socket_W", "power_cap_W", "GiB_per_s", "gfxclk_MHz_median")
        mine = [float(power.get(k) or -1.0) for k in keys]
        allp = shard.gather_floats(mine, world, group)
        if world > 1:
            power = {"per_gpu": [dict(rank=r, **{k: (v if v >= 0 else None) for k, v in zip(keys, row)})
                                 for r, row in enumerate(allp)],
                     "method": power.get("method") if isinstance(power, dict) else None}
        phase("power_s")

    line = None
    if rank == 0:
        all_dig = res["digests"]
        wall_max, kern_max = res["wall_max"], res["kernel_ms_max"]
        total_bytes = world * C * CHUNK * args.steps
        value = total_bytes / wall_max / 2**30
        bytes_per_launch = C * CHUNK
        achieved = bytes_per_launch / (kern_max * 1e-3) / 1e9
        valu_tops = C * (CHUNK // 64 + 1) * VALU_OPS_PER_BLOCK / (kern_max * 1e-3) / 1e12

        # Parity spot check of the timed output: global chunks 0..4095 are the
        # committed golden vectors (tests/golden/synth4096.txt, from sha.c).
        parity = None
        golden = os.path.join(HERE, "tests", "golden", "synth4096.txt")
        if os.path.exists(golden) and world * C >= 4096:
            rows = [l.split() for l in open(golden) if not l.startswith("#")]
            parity = all(all_dig[20 * int(i):20 * int(i) + 20].hex() == h for i, h in rows)

        # A few digests of every rank (first, last and evenly between), by
        # GLOBAL chunk index: the tests recompute them with the oracle on
        # regenerated chunks, covering ranks >= 1 beyond the golden range.
        sample = None
        if args.digest_sample > 0:
            sample = [{"rank": r, "chunk": g, "sha1": all_dig[20 * g:20 * g + 20].hex()}
                      for r, g in shard.sample_chunks(world, C, args.digest_sample)]

        # A checksum of ALL digests in global chunk order (SHA-1 of the
        # concatenated 20-byte digests, hashlib): the tests compare it with the
        # oracle's digests of every regenerated chunk of every rank.
        import hashlib
        digests_sha1 = hashlib.sha1(all_dig).hexdigest() if all_dig else None
        # ... and against the REFERENCE's checksum for this many global chunks
        # (tests/golden/synth_checksums.txt, sha.c's digests of the same
        # chunks): every digest of the run, every rank, in one comparison.
        parity_all = None
        sums = os.path.join(HERE, "tests", "golden", "synth_checksums.txt")
        if digests_sha1 and os.path.exists(sums):
            table = dict(l.split() for l in open(sums) if l.strip() and not l.startswith("#"))
            if str(world * C) in table:
                parity_all = table[str(world * C)] == digests_sha1

        # PMC traffic, only when measured on this very build and layout.
        want = {"chunks": C, "pitch": pitch, "source_id": bt.source_id(), "kernel": kernel,
                "variant": bt.build_info().split("ring=")[1].split()[0]}
        traffic, traffic_note = find_traffic(want, args.traffic_json)
        phase("gather_and_parity_s")

        # Rank 0 runs the CPU baseline at every N (the other ranks wait at the
        # final barrier, their GPUs idle): each line carries the reference
        # sha.c on this node's host cores from the same run (north_star).
        # The host paths (config 5) are a one-GPU measurement (N = 1 only).
        want_host = world == 1 and not args.no_host_path
        extras_host = None
        if not args.no_cpu_baseline or want_host:
            import numpy as np
            n_host = min(C, max(args.cpu_chunks if not args.no_cpu_baseline else 0,
                                int(args.host_gib * 2**30) // CHUNK if want_host else 0))
            extras_host = np.empty(n_host * CHUNK, dtype=np.uint8)
            view = torch.from_numpy(extras_host)
            for i in range(0, n_host, 2048):  # 1 GiB slices
                k = min(2048, n_host - i)
                if pitch == CHUNK:
                    view[i * CHUNK:(i + k) * CHUNK].copy_(hasher.buf[i * CHUNK:(i + k) * CHUNK])
                else:
                    for j in range(i, i + k):
                        view[j * CHUNK:(j + 1) * CHUNK].copy_(hasher.buf[j * pitch:j * pitch + CHUNK])

        cpu = None
        if not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(extras_host.ctypes.data, min(args.cpu_chunks, C), all_dig)
            except Exception as e:  # the checker must never cost the bench line
                cpu = {"error": f"{type(e).__name__}: {e}"}
            phase("cpu_baseline_s")

        verify = None
        if world == 1:
            try:
                verify = hasher.verify_rate()
            except Exception as e:  # noqa: BLE001 -- never costs the bench line
                verify = {"error": f"{type(e).__name__}: {e}"}
            phase("verify_dev_s")

        host = None
        if want_host and pitch == CHUNK:
            try:
                n_img = min(C, int(args.host_gib * 2**30) // CHUNK)
                host = host_paths(bt, torch, hasher.buf, extras_host[:n_img * CHUNK], all_dig[:20 * n_img])
            except Exception as e:
                host = {"error": f"{type(e).__name__}: {e}"}
            phase("host_path_s")

        peak_at_clock = (VALU_MIX_PEAK_TOPS * (clock["in_kernel_mhz"] / 1000.0 / CLOCK_GHZ)
                         if clock and "in_kernel_mhz" in clock else None)
        line = {
            "metric": METRIC,
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
                "build": bt.build_info(),
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": kernel, "kernel_ms": round(kern_max, 4),
                "kernel_ms_median_rank0": round(hasher.kernel_ms_median(), 4),
                "algorithmic_bytes_per_launch": bytes_per_launch, "traffic_source": traffic_note,
            },
            "valu_roofline": None if kernel != "k_sha1_fixed" else {
                "bound": "valu", "achieved": round(valu_tops, 2), "unit": "T int32 lane-ops/s",
                "peak": round(VALU_MIX_PEAK_TOPS, 2), "frac": round(valu_tops / VALU_MIX_PEAK_TOPS, 4),
                "peak_at_measured_clock": round(peak_at_clock, 2) if peak_at_clock else None,
                "frac_at_measured_clock": round(valu_tops / peak_at_clock, 4) if peak_at_clock else None,
                "ops_per_block": VALU_OPS_PER_BLOCK,
                "peak_basis": f"{VALU_OPS_PER_BLOCK}-op mix ({VALU_HALF_RATE_PER_BLOCK} half-rate) on 1024 SIMDs "
                              "at 2.4 GHz / at the in-kernel clock"},
            "clock": clock,
            "power": power,
            # per rank: its rate and kernel time, and which GPU it was (PCI address,
            # UUID, devices visible), which kernel it ran and on which global chunks
            "per_gpu": [{**idents[r], "GiB_per_s": round(C * CHUNK * args.steps / w / 2**30, 3),
                         "kernel_ms": round(k, 4), "kernel_GiB_per_s": round(C * CHUNK / (k * 1e-3) / 2**30, 3),
                         "in_kernel_mhz": rank_mhz[r] if rank_mhz else None}
                        for r, (w, k) in enumerate(res["per_rank"])],
            # SURVEY.md §8d config 4's aggregate: all ranks' bytes of one step /
            # the slowest rank's average hot-kernel time (HIP events)
            "aggregate_kernel_GiB_per_s": round(world * C * CHUNK / (kern_max * 1e-3) / 2**30, 3),
            "distinct_gpus": shard.distinct_devices(idents),
            "rehearse_shared_gpu": bool(args.rehearse_shared_gpu),
            "parity_first_4096_vs_golden": parity,
            "digest_sample": sample,
            "digests_sha1": digests_sha1,
            "parity_all_vs_golden": parity_all,
            "cpu_baseline": cpu,
            "verify_dev": verify,
            "host_path": host,
            "phases_s": phases,
            # this process's age when the line is printed (interpreter start -> print)
            "bench_wall_s": process_age_s(),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        shard.barrier(world, group)
        dist.destroy_process_group()
    return line


shard = _load("shard", os.path.join(PKG, "shard.py"))

if __name__ == "__main__":
    main()
