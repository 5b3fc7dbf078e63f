"""GPU: bench.py's own multi-rank path, launched exactly as the driver launches
it for N > 1 (torch.distributed.run, one process per rank, 127.0.0.1
rendezvous), with every rank on this box's one MI355X (8 ranks = the driver's N = 8 line).

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


def _run_bench(world, chunks, *extra, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(world), "--chunks", str(chunks),
           "--steps", "3", "--warmup", "1", *extra]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints the line
    return json.loads(lines[0])


def _check_identity(line, world, chunks):
    """Every per_gpu entry says which GPU the rank drove (PCI address, UUID,
    devices visible), which kernel it ran and on which global chunks.  All
    ranks share this box's one GPU, so the addresses are equal and the
    distinct-device guard stays off (device_count 1 < world)."""
    per = line["per_gpu"]
    assert [p["rank"] for p in per] == list(range(world))
    for r, p in enumerate(per):
        for k in ("pci_bdf", "uuid", "device_count", "hip_device", "kernel", "chunk_range"):
            assert k in p, (k, p)
        assert p["kernel"] == line["roofline"]["kernel"]
        assert p["chunk_range"] == [r * chunks, (r + 1) * chunks]
        assert p["device_count"] >= 1 and len(p["pci_bdf"].split(":")) == 3
    assert len({p["pci_bdf"] for p in per}) == line["distinct_gpus"]
    if per[0]["device_count"] < world:
        assert line["distinct_gpus"] == 1 and len({p["uuid"] for p in per}) == 1


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
    line = _run_bench(world, chunks)
    assert line["n_gpus"] == world and line["steps"] == 3 and line["warmup"] == 1
    assert line["config"]["global_chunks"] == 4096
    assert line["parity_first_4096_vs_golden"] is True
    assert [p["rank"] for p in line["per_gpu"]] == list(range(world))
    assert all(p["GiB_per_s"] > 0 and p["kernel_ms"] > 0 for p in line["per_gpu"])
    assert line["value"] > 0 and line["scaling"] == "weak"
    # N > 1: no CPU baseline / host-path legs (rank 0 at N = 1 only)
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
    line = _run_bench(world, chunks, "--power-s", "0", timeout=300)
    assert line["roofline"]["kernel"] == "k_sha1_fixed"
    assert line["config"]["global_chunks"] == world * chunks
    assert line["parity_first_4096_vs_golden"] is True   # rank 0's first 4096 vs sha.c golden
    assert [p["rank"] for p in line["per_gpu"]] == list(range(world))
    _check_identity(line, world, chunks)
    _check_sample(line, world, chunks, oracle)


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
    _check_sample(line, 1, 4096, oracle)
