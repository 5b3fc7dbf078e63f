"""GPU: bench.py's own multi-rank path, launched exactly as the driver launches
it for N > 1 (torch.distributed.run, one process per rank, 127.0.0.1
rendezvous) and as a plain `python bench.py --gpus N` (bench.py then starts
the ranks itself), with every rank on this box's one MI355X (8 ranks = the
driver's N = 8 line) under --rehearse-shared-gpu -- and refused without it.

What runs is the code the 8-GPU scaling bench runs: DeviceHasher per rank
(device generator over the rank's GLOBAL chunk range, one launch per step of the
kernel the per-rank batch size selects),
shard.run_rank (barriers, max-over-ranks timing, host-side digest gather on
the gloo control plane).  The ranks together hash global chunks 0..4095, so
rank 0's `parity_first_4096_vs_golden` checks every rank's digests AND the
gather order against the reference's golden vectors (tests/golden/synth4096.txt,
produced by sha.c) -- config 4's split at a size one GPU holds.

Those per-rank sizes (512..2048 chunks) select the latency kernels, so the
second test runs the rank path at a per-rank size that selects the HOT kernel
(k_sha1_fixed, > 128 chunks per CU): 2 ranks x 40960 chunks (2 x 20 GiB on the
one MI355X) and 2 ranks x 131072 chunks (config 4's exact per-rank size), with the line's `digest_sample` -- first, middle and last chunk of
EVERY rank by global index -- recomputed by the oracle on regenerated chunks,
so rank 1's chunks 40960..81919 (far past the golden range) are checked too;
and the line's `digests_sha1` (a checksum of ALL gathered digests in global
order) is compared with the oracle's digests of every chunk of every rank.
chunk.c:20-21 carries no state between chunks, hence the contiguous split.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu
CHUNK = 512 * 1024


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_bench(world, chunks, *extra, timeout=240, launcher=True, shared=True):
    """bench.py at `world` ranks on this box's one GPU: launched the driver's
    N > 1 way (torch.distributed.run) or, launcher=False, as the plain
    `python bench.py --gpus N` the driver may also run (bench.py starts the
    ranks itself).  All ranks share the one GPU, so the run needs
    --rehearse-shared-gpu (shared=True); without it bench.py must refuse."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    if not shared:
        # every rank on ONE device even on a box that shows several: the first
        # of the devices this process may use
        vis = env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES")
        env["HIP_VISIBLE_DEVICES"] = vis.split(",")[0] if vis else "0"
    args = [os.path.join(REPO, "bench.py"), "--gpus", str(world), "--chunks", str(chunks),
            "--steps", "3", "--warmup", "1", *extra] + (["--rehearse-shared-gpu"] if shared else [])
    if launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    if not shared:
        return r
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints the line
    return json.loads(lines[0])


def _check_identity(line, world, chunks):
    """Every per_gpu entry says which GPU the rank drove (host, PCI address,
    UUID, devices visible), which kernel it ran and on which global chunks.
    All ranks share this box's one GPU, so the identities are equal, and the
    line says the rank path was rehearsed on a shared GPU on purpose."""
    per = line["per_gpu"]
    assert [p["rank"] for p in per] == list(range(world))
    for r, p in enumerate(per):
        for k in ("host", "pci_bdf", "uuid", "device_count", "hip_device", "kernel", "chunk_range"):
            assert k in p, (k, p)
        assert p["kernel"] == line["roofline"]["kernel"]
        assert p["chunk_range"] == [r * chunks, (r + 1) * chunks]
        assert p["device_count"] >= 1 and len(p["pci_bdf"].split(":")) == 3
    assert len({(p["host"], p["pci_bdf"], p["uuid"]) for p in per}) == line["distinct_gpus"]
    if per[0]["device_count"] < world:
        assert line["distinct_gpus"] == 1 and len({p["uuid"] for p in per}) == 1
    assert line["rehearse_shared_gpu"] is (world > 1)


def _check_sample(line, world, chunks, oracle):
    """Every rank's sampled digests == the oracle on the regenerated chunk."""
    sample = line["digest_sample"]
    assert sorted({s["rank"] for s in sample}) == list(range(world))
    for r in range(world):
        got = sorted(s["chunk"] for s in sample if s["rank"] == r)
        assert got[0] == r * chunks and got[-1] == (r + 1) * chunks - 1, got
    for s in sample:
        data = bytes(oracle.fill_synthetic(CHUNK, s["chunk"] * (CHUNK // 8), oracle.SEED_SYNTH))
        assert oracle.sha1(data).hex() == s["sha1"], s
    # every digest of every rank, gathered in global order: the line's checksum
    # of all of them == the oracle's over every regenerated chunk
    want = oracle.synth_digests(0, world * chunks)
    assert hashlib.sha1(want).hexdigest() == line["digests_sha1"]
    # and bench.py's own comparison with the reference's checksum for this
    # global chunk count (tests/golden/synth_checksums.txt, from sha.c)
    assert line["parity_all_vs_golden"] is True


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_ranks_split_and_gather_on_one_gpu(world, oracle):
    chunks = 4096 // world
    line = _run_bench(world, chunks, "--no-cpu-baseline")
    assert line["n_gpus"] == world and line["steps"] == 3 and line["warmup"] == 1
    assert line["config"]["global_chunks"] == 4096
    assert line["parity_first_4096_vs_golden"] is True
    assert [p["rank"] for p in line["per_gpu"]] == list(range(world))
    assert all(p["GiB_per_s"] > 0 and p["kernel_ms"] > 0 for p in line["per_gpu"])
    # §8d config 4's aggregate: all ranks' bytes / the slowest rank's kernel time
    slowest = max(p["kernel_ms"] for p in line["per_gpu"])
    assert abs(line["aggregate_kernel_GiB_per_s"] - world * chunks * CHUNK / (slowest * 1e-3) / 2**30) < \
        1e-3 * line["aggregate_kernel_GiB_per_s"] + 0.01
    assert all(abs(p["kernel_GiB_per_s"] * p["kernel_ms"] * 1e-3 * 2**30 - chunks * CHUNK) < 1e-3 * chunks * CHUNK
               for p in line["per_gpu"])
    assert line["value"] > 0 and line["scaling"] == "weak"
    # N > 1: no host-path leg (rank 0 at N = 1 only); the CPU baseline was
    # switched off here (test_bench_gpus_flag_alone_starts_the_ranks runs it)
    assert line["cpu_baseline"] is None and line["host_path"] is None
    # every rank read its own GPU's board power after the timed region
    assert [p["rank"] for p in line["power"]["per_gpu"]] == list(range(world))
    _check_identity(line, world, chunks)
    _check_sample(line, world, chunks, oracle)


@pytest.mark.parametrize("world,chunks", [(2, 40960), (2, 131072), (8, 40960)])
def test_bench_ranks_run_the_hot_kernel_with_parity_on_every_rank(oracle, world, chunks):
    """Config 4's per-rank kernel through the rank path: at 40960 chunks per
    rank the batch selects k_sha1_fixed (one-wave workgroups, < 1 wave per
    SIMD), and 131072 per rank is exactly the 8-GPU bench's per-rank workload
    (64 GiB each, 128 GiB for both ranks in the one GPU's 288 GB).  Eight
    ranks x 40960 (160 GiB on the one GPU) is the driver's N = 8 launch with
    every rank on the hot kernel: 327,680 digests, all compared with the
    reference's checksum and with the oracle."""
    line = _run_bench(world, chunks, "--power-s", "0", "--no-cpu-baseline", timeout=300)
    assert line["roofline"]["kernel"] == "k_sha1_fixed"
    assert line["config"]["global_chunks"] == world * chunks
    assert line["parity_first_4096_vs_golden"] is True   # rank 0's first 4096 vs sha.c golden
    assert [p["rank"] for p in line["per_gpu"]] == list(range(world))
    _check_identity(line, world, chunks)
    _check_sample(line, world, chunks, oracle)
    _check_rank_clocks(line, world)


def _check_rank_clocks(line, world):
    """Every rank stamped its own in-kernel clock after the timed region; the
    VALU roofline is priced at the slowest rank's."""
    mhz = [p["in_kernel_mhz"] for p in line["per_gpu"]]
    assert all(m is not None and 300 < m < 3000 for m in mhz), mhz
    clock = line["clock"]
    assert clock["in_kernel_mhz"] == min(mhz) and clock["probe_digests_identical"] is True
    assert clock["per_rank_mhz"] == mhz and mhz[clock["slowest_rank"]] == min(mhz)
    v = line["valu_roofline"]
    assert abs(v["peak_at_measured_clock"] - v["peak"] * min(mhz) / 2400.0) < 0.02 * v["peak"]


@pytest.mark.parametrize("world,chunks", [(2, 40960), (8, 512)])
def test_bench_gpus_flag_alone_starts_the_ranks(oracle, world, chunks):
    """`python3 bench.py --gpus N` with no launcher (the driver's BENCH command
    shape): bench.py starts the N ranks itself and relays rank 0's one line
    -- n_gpus N, N per_gpu entries, every digest equal to the reference's
    checksum (81,920 chunks on the hot kernel with per-rank clocks; 8 ranks x
    512 chunks = config 2's 4096 on the latency kernel) -- and, as every
    N > 1 SCALE line must (north_star: "next to the reference sha.c timed on
    the GPU box's own host cores in the same run"), rank 0's CPU baseline:
    the reference's own sha.c, its digests equal to the GPU's."""
    line = _run_bench(world, chunks, "--power-s", "0", launcher=False, timeout=300)
    assert line["n_gpus"] == world and len(line["per_gpu"]) == world
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "reference" and cpu["digests_match_gpu"] is True, cpu
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and "O2_1t" in cpu["runs"]
    assert line["host_path"] is None and line["phases_s"]["cpu_baseline_s"] > 0
    assert line["config"]["global_chunks"] == world * chunks
    assert line["parity_all_vs_golden"] is True and line["parity_first_4096_vs_golden"] is True
    _check_identity(line, world, chunks)
    if line["roofline"]["kernel"] == "k_sha1_fixed":
        _check_rank_clocks(line, world)
    else:  # the probe stamps the hot kernel only
        assert line["clock"] is None and all(p["in_kernel_mhz"] is None for p in line["per_gpu"])


@pytest.mark.parametrize("launcher", [True, False])
def test_bench_refuses_ranks_sharing_a_gpu_without_the_rehearsal_flag(launcher):
    """Two ranks on this box's one GPU without --rehearse-shared-gpu: every
    rank exits before the timed region (a line claiming 2 GPUs on 1 is never
    printed), whichever way the ranks were started."""
    r = _run_bench(2, 512, "--power-s", "0", "--no-clock", launcher=launcher, shared=False, timeout=240)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "distinct GPU" in r.stderr and "--rehearse-shared-gpu" in r.stderr


def test_bench_single_rank_line_checks(oracle):
    """bench.py at N = 1 (plain `python bench.py`, as the driver runs it) at
    config 2's 4096 chunks: parity against the reference's golden digests and
    checksum, and the device-resident verify leg flags exactly the planted
    mismatches (the fused compare of util.c:311-313)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--chunks", "4096", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--no-host-path", "--power-s", "0"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["parity_first_4096_vs_golden"] is True
    assert line["parity_all_vs_golden"] is True
    _check_identity(line, 1, 4096)
    assert 0 < line["bench_wall_s"] < 600 and line["phases_s"]["warmup_and_timed_s"] > 0
    v = line["verify_dev"]
    assert v["flags_correct"] is True and v["mismatches_planted"] == len(range(0, 4096, 997)) and v["GiB_per_s"] > 0
    # the fused compare, timed paired with the plain hash in one window
    assert v["hash_ms"] > 0 and v["verify_ms"] > 0 and v["pairs"] >= 5
    assert abs(v["overhead_pct"] - 100.0 * (v["verify_ms"] / v["hash_ms"] - 1.0)) < 0.01
    o = v["overhead_pct_pairs"]
    assert o["min"] <= o["median"] <= o["max"]
    assert line["rehearse_shared_gpu"] is False and line["distinct_gpus"] == 1
    _check_sample(line, 1, 4096, oracle)


def test_bench_host_path_leg_explains_itself(oracle):
    """Config 5 in the N = 1 line (a 1 GiB image here): each pipeline rate is
    the median of 5 steady-state runs after a first one, every run listed
    with its phase split (providing the input on the host vs blocked on the
    GPU lane, page registration), machine CPU load and cgroup throttling;
    the pageable image is fed both ways -- page-locked batch by batch (the
    default) and copied into the staging lanes -- each with its NUMA
    placement; the batched verifier is fed zero-copy and packetized
    (util.c:275's 1484-byte memcpys) on one and on four receive threads --
    every digest and verdict right."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--chunks", "4096", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--host-gib", "1", "--power-s", "0", "--no-clock"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    hp = line["host_path"]
    assert hp["image_GiB"] == 1.0
    assert hp["fields"] and len(json.dumps(line)) < 8000  # the whole line stays compact
    for key in ("pageable_chunks_host", "pageable_staged_copy", "registered_direct_dma"):
        p = hp[key]
        runs = p["runs_GiB_per_s"]
        assert p["digests_match"] is True and len(runs) == 6, p
        assert p["GiB_per_s"] == round(sorted(runs[1:])[2], 3) and p["first_run_GiB_per_s"] == runs[0]
        for run in (p["median_run"], p.get("first_run", p["median_run"])):
            assert run["s"] > 0 and run["wait_s"] >= 0 and run["fill_s"] >= 0
            assert run["fill_s"] + run["wait_s"] <= run["s"] * 1.05 + 1e-3
        m = p["median_run"]
        assert m["cpu_s"] >= 0 and 0 <= m["fill_frac"] <= 1.05 and m["lock_s"] >= 0 and m["unlock_s"] >= 0
        assert 0 < p["frac_of_raw_h2d"] < 1.2
    reg, stg = hp["pageable_chunks_host"]["numa"], hp["pageable_staged_copy"]["numa"]
    assert reg["feed"] == "registered" and reg["locked_batches"] == [2, 2] and sum(reg["staging_pieces"]) == 0
    # the last 1024 of 2048 chunks go by columns (1023 when the image's last
    # page is partial: that chunk is hashed from a pinned copy); 2 x 256 MiB batches
    assert reg["column_chunks"] in (1023, 1024)
    assert stg["feed"] == "staged" and stg["locked_batches"] == [0, 2]
    assert sum(stg["image_pages"]) > 0 and sum(stg["lane_pages"]) > 0 and sum(stg["staging_pieces"]) > 0
    assert len(stg["image_pages"]) == len(stg["lane_pages"]) == len(stg["staging_pieces"]) >= 1
    if stg["policy"] in ("lanes", "gpu"):  # the lanes sit on the GPU's node
        assert stg["lane_pages"][stg["gpu_node"]] == sum(stg["lane_pages"])
    for key, threads in (("zero_copy_verifier", 1), ("packetized_verifier", 1), ("packetized_verifier_4_threads", 4)):
        v = hp[key]
        assert v["digests_match"] is True and v["GiB_per_s"] > 0 and "error" not in v, (key, v)
        assert v["receive_threads"] == threads and v["args"]
    assert hp["packetized_verifier"]["timed_chunks"] == 2 * 2048
