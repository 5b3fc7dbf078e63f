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
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_ranks_split_and_gather_on_one_gpu(world):
    chunks = 4096 // world
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(world), "--chunks", str(chunks),
           "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints the line
    line = json.loads(lines[0])
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
