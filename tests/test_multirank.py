"""CPU, world_size 2 (gloo): the multi-GPU split and the host-side digest
gather produce exactly the single-process digests in global chunk order.
The per-rank hashing here is the oracle standing in for the kernel (no GPU
in this container); the partition / gather code is the product's (shard.py,
the same logic bench.py and bt_sha1_chunks_host_multi use)."""
import importlib.util
import os
import socket

import pytest
import torch.multiprocessing as mp

from conftest import PKG, REPO, read_pairs

CHUNK = 4096  # small chunks keep the CPU oracle fast


def _load_shard():
    spec = importlib.util.spec_from_file_location("shard", os.path.join(PKG, "shard.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, q):
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import py_oracle
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = _load_shard()
    if mode == "weak":
        lo, hi = shard.weak_range(rank, 5)
        data = py_oracle.fill_synthetic((hi - lo) * CHUNK, lo * (CHUNK // 8), py_oracle.SEED_SYNTH)
        local = b"".join(py_oracle.hash_chunks(data, CHUNK))
    else:  # strong split of one 37-chunk image with a short tail
        n_bytes = 36 * CHUNK + 1234
        n = (n_bytes + CHUNK - 1) // CHUNK
        lo, hi = shard.block_range(n, world, rank)
        img = py_oracle.fill_synthetic(n_bytes, 0, 77)
        local = b"".join(py_oracle.hash_chunks(bytes(img[lo * CHUNK:min(hi * CHUNK, n_bytes)]), CHUNK))
    out = shard.gather_digests(local, world, rank)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


class StubHasher:
    """CPU stand-in for bench.DeviceHasher (same protocol: step/sync/kernel_ms/
    digests); the hashing is the oracle on small chunks."""

    def __init__(self, oracle, first_chunk, chunks):
        self.oracle, self.first, self.C = oracle, first_chunk, chunks
        self.data = oracle.fill_synthetic(chunks * CHUNK, first_chunk * (CHUNK // 8), oracle.SEED_SYNTH)
        self.steps, self.out = [], b""

    def step(self, i):
        self.steps.append(i)
        self.out = b"".join(self.oracle.hash_chunks(self.data, CHUNK))

    def sync(self):
        pass

    def kernel_ms(self):
        return 1.0 + self.first / 1000.0  # distinct per rank: the max must pick the last rank

    def digests(self):
        return self.out


def _bench_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import py_oracle
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = _load_shard()
    C = 6
    lo, _ = shard.weak_range(rank, C)
    h = StubHasher(py_oracle, lo, C)
    res = shard.run_rank(h, steps=4, warmup=2, world=world, rank=rank)
    assert h.steps == [-1, -2, 0, 1, 2, 3]
    # the distinct-device exchange of the same launch: one GPU per rank on one node
    ident = {"rank": rank, "host": "node0", "pci_bdf": f"0000:{0x05 + 0x10 * rank:02x}:00.0", "uuid": f"u{rank}"}
    idents = shard.gather_objects(ident, world)
    assert shard.check_distinct_devices(idents, world) is None and shard.distinct_devices(idents) == world
    if rank == 0:
        q.put((res["digests"], res["kernel_ms_max"], len(res["per_rank"])))
    else:
        assert res["digests"] is None
    shard.barrier(world)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_bench_rank_protocol(oracle, world):
    """bench.py's own per-rank protocol (shard.run_rank: warmup, barriers,
    timed steps, max over ranks, ordered digest gather, and the pre-timing
    identity exchange) with a CPU stub hasher, at world size 2 and at config
    4's 8 ranks: rank 0 ends up with all 6 x world digests in global order and
    the slowest rank's kernel time."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    dig, kmax, nranks = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = b"".join(oracle.hash_chunks(oracle.fill_synthetic(6 * world * CHUNK, 0, oracle.SEED_SYNTH), CHUNK))
    assert dig == want
    assert nranks == world and abs(kmax - (1.0 + 6 * (world - 1) / 1000.0)) < 1e-9


def _ident_worker(rank, world, port, shared, allow, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = _load_shard()
    bdf = "0000:05:00.0" if shared else f"0000:{0x05 + 0x10 * rank:02x}:00.0"
    # shared: the one-GPU box (device_count 1, one PCI address for both ranks)
    ident = {"rank": rank, "host": "box", "pci_bdf": bdf, "uuid": "stub-0" if shared else f"stub-{rank}",
             "device_count": 1 if shared else world,
             "kernel": "k_sha1_fixed", "chunk_range": list(shard.weak_range(rank, 131072))}
    idents = shard.gather_objects(ident, world)
    q.put((rank, idents, shard.check_distinct_devices(idents, world, allow_shared=allow),
           shard.distinct_devices(idents)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("shared,allow", [(False, False), (True, False), (True, True)])
def test_rank_identities_gathered_and_shared_gpu_refused(shared, allow):
    """bench.py's pre-timing identity exchange at world size 2 (gloo): every
    rank gets every rank's {host, PCI address, UUID, devices visible, kernel,
    chunk range} in rank order.  Two ranks on one GPU -- here a stub pair on
    one PCI address with device_count 1, the shape of a one-GPU box -- give
    EVERY rank the clash (all exit before the timed region) unless the launch
    asked for a shared-GPU rehearsal (--rehearse-shared-gpu)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ident_worker, args=(r, world, port, shared, allow, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, idents, clash, distinct in got:
        assert [i["rank"] for i in idents] == [0, 1]
        assert [i["chunk_range"] for i in idents] == [[0, 131072], [131072, 262144]]
        assert distinct == (1 if shared else 2)
        if shared and not allow:
            assert clash and "0000:05:00 on box <- ranks [0, 1]" in clash and "--rehearse-shared-gpu" in clash
        else:
            assert clash is None


def test_distinct_device_guard_logic():
    shard = _load_shard()

    def ids(bdfs, count, hosts=None):
        return [{"rank": r, "host": (hosts or ["n0"] * len(bdfs))[r], "pci_bdf": b, "uuid": None,
                 "device_count": count} for r, b in enumerate(bdfs)]
    full = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xe5, 0xf5)]
    assert shard.check_distinct_devices(ids(full, 8), 8) is None            # a full node, one GPU per rank
    assert shard.check_distinct_devices(ids(full, 1), 8) is None            # one visible device per rank, distinct
    bad = full[:7] + [full[3]]
    msg = shard.check_distinct_devices(ids(bad, 8), 8)
    assert msg and "ranks [3, 7]" in msg and "7 distinct" in msg            # two ranks on one GPU
    assert shard.check_distinct_devices(ids(bad, 1), 8)                     # ... whatever device_count says
    assert shard.check_distinct_devices(ids([full[0]] * 8, 1), 8)           # one-GPU box: refused by default
    assert shard.check_distinct_devices(ids([full[0]] * 8, 1), 8, allow_shared=True) is None  # the rehearsal
    assert shard.check_distinct_devices(ids([full[0]] * 2, 1), 2)
    assert "4 of 8" in shard.check_distinct_devices(ids(full[:4], 4), 8)    # incomplete gather
    assert shard.check_distinct_devices(ids(full[:1], 8), 1) is None        # N = 1
    # two nodes x 4 ranks: equal PCI addresses on different hosts are different GPUs
    two = ids(full[:4] * 2, 8, hosts=["n0"] * 4 + ["n1"] * 4)
    assert shard.check_distinct_devices(two, 8) is None and shard.distinct_devices(two) == 8
    # UUIDs from one source only split keys: same address + host, different UUIDs -> distinct
    parts = [{"rank": r, "host": "n0", "pci_bdf": full[0], "uuid": f"u{r}", "uuid_source": "smi"} for r in range(2)]
    assert shard.check_distinct_devices(parts, 2) is None


def _smi_ident(rank, smi_bdf, uuid="54ff75a3-0000-1000-806c-9eb5603801dc", hip_bdf=None):
    """A rank whose amdsmi lookup worked: amdsmi's full address (with the
    function number) beside HIP's (function fixed at .0), amdsmi's UUID."""
    return {"rank": rank, "host": "n0", "pci_bdf": hip_bdf or smi_bdf.rsplit(".", 1)[0] + ".0",
            "smi_bdf": smi_bdf, "uuid": uuid, "uuid_source": "smi", "device_count": 1}


def test_gpu_identity_keys_on_the_full_pci_address():
    """Partitions of one GPU differ only in the PCI function number, which HIP
    does not report (bench.py builds pci_bdf with .0): with amdsmi's address
    on every rank, ...:00.0 and ...:00.1 are two devices, and two ranks at one
    smi_bdf are refused.  Spellings are normalised (case, domain)."""
    shard = _load_shard()
    two = [_smi_ident(0, "0000:5d:00.0", "u-a"), _smi_ident(1, "0000:5d:00.1", "u-b")]
    assert two[0]["pci_bdf"] == two[1]["pci_bdf"] == "0000:5d:00.0"
    assert shard.check_distinct_devices(two, 2) is None and shard.distinct_devices(two) == 2
    # the same UUID (one physical package) does not merge two functions either
    same_pkg = [_smi_ident(0, "0000:5d:00.0"), _smi_ident(1, "0000:5d:00.1")]
    assert shard.check_distinct_devices(same_pkg, 2) is None
    one = [_smi_ident(0, "0000:5d:00.1"), _smi_ident(1, "0000:5D:00.1")]
    msg = shard.check_distinct_devices(one, 2)
    assert msg and "0000:5d:00.1 on n0 <- ranks [0, 1]" in msg and shard.distinct_devices(one) == 1


def test_gpu_identity_never_splits_one_gpu_over_two_sources():
    """amdsmi and HIP spell one GPU's UUID differently, and only
    amdsmi gives the function number.  A launch where amdsmi failed on some
    ranks of a shared GPU must still be refused: every rank is then keyed on
    the coarser address (domain:bus:device) and no UUID."""
    shard = _load_shard()
    smi = _smi_ident(0, "0000:5d:00.0")
    hip = {"rank": 1, "host": "n0", "pci_bdf": "0000:5d:00.0", "uuid": "GPU-9eb5603801dc", "uuid_source": "hip",
           "smi_error": "AmdSmiLibraryException", "device_count": 1}
    msg = shard.check_distinct_devices([smi, hip], 2)
    assert msg and "ranks [0, 1]" in msg and shard.distinct_devices([smi, hip]) == 1
    # ... also when the amdsmi rank sits on function 1 of the same device
    smi1 = _smi_ident(0, "0000:5d:00.1")
    assert shard.check_distinct_devices([smi1, hip], 2)
    # both ranks on HIP's fields alone: one source, so its UUIDs may split
    hip0 = dict(hip, rank=0, uuid="GPU-a")
    assert shard.check_distinct_devices([hip0, hip], 2) is None
    assert shard.check_distinct_devices([hip0, dict(hip, uuid="GPU-a")], 2)
    # distinct GPUs stay distinct under the coarse key
    other = dict(hip, pci_bdf="0000:75:00.0")
    assert shard.check_distinct_devices([smi, other], 2) is None


def test_bench_uses_the_shard_protocol():
    """The bench's rank split / timing / gather is shard.py's (covered above),
    not an inline copy."""
    src = open(os.path.join(REPO, "bench.py")).read()
    assert "shard.run_rank(" in src and "shard.weak_range(" in src
    assert "dist.gather(" not in src and "dist.all_gather(" not in src


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_two_rank_split_equals_single(mode, oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if mode == "weak":
        data = oracle.fill_synthetic(10 * CHUNK, 0, oracle.SEED_SYNTH)
        want = b"".join(oracle.hash_chunks(data, CHUNK))
    else:
        img = oracle.fill_synthetic(36 * CHUNK + 1234, 0, 77)
        want = b"".join(oracle.hash_chunks(bytes(img), CHUNK))
    assert got == want


def test_block_range_covers_exactly():
    shard = _load_shard()
    for n in [0, 1, 7, 8, 131072, 1048576]:
        for world in [1, 2, 4, 8]:
            rs = [shard.block_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
    # weak scaling at 8 GPUs = BASELINE config 4's 1 M chunks
    assert shard.weak_range(7, 131072) == (917504, 1048576)


def test_digest_sample_covers_every_rank_edges():
    """bench.py's digest_sample picks: first and last chunk of EVERY rank (so
    ranks >= 1, beyond the golden range, are checked), evenly between."""
    shard = _load_shard()
    got = shard.sample_chunks(8, 131072, 3)
    assert [r for r, _ in got] == [r for r in range(8) for _ in range(3)]
    for r in range(8):
        mine = [g for rr, g in got if rr == r]
        assert mine == [r * 131072, r * 131072 + 65535, (r + 1) * 131072 - 1]
    assert shard.sample_chunks(2, 1, 3) == [(0, 0), (1, 1)]  # one chunk per rank: no duplicates
    assert shard.sample_chunks(2, 5, 0) == []


def test_bench_cpu_baseline_leg(oracle):
    """bench.py's cpu_baseline leg on CPU: sustained medians, `cores` = the
    usable CPU budget (affinity capped by the cgroup quota), thread counts
    reported separately, and the reference's digests compared with the
    (here: oracle-made) device digests."""
    import ctypes
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    n, chunk = 8, 512 * 1024
    data = bytes(oracle.fill_synthetic(n * chunk, 0, oracle.SEED_SYNTH))
    buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
    want = b"".join(oracle.hash_chunks(data, chunk))
    cb = bench.cpu_baseline(ctypes.addressof(buf), n, want, min_s=0.05, reps=2)
    cores, _, quota = bench.usable_cores()
    assert cb["cores"] == cores
    assert cb["kind"] in ("reference", "port") and cb["digests_match_gpu"] is True
    multi = [r for k, r in cb["runs"].items() if k.startswith("O2_") and r["threads"] > 1]
    if multi:  # the best multi-thread -O2 run, its thread count reported beside `cores`
        best = max(multi, key=lambda r: r["GiB_per_s"])
        assert cb["value"] == best["GiB_per_s"] > 0 and cb["threads"] == best["threads"]
        assert f"O2_{cores}t" in cb["runs"]
    assert {"O2_1t", "O0_1t"} <= set(cb["runs"]) and cb["per_core_GiB_per_s_O2"] > 0
    assert all(r["passes"] >= 2 for r in cb["runs"].values())  # repeated until >= min_s, twice
    assert cb["runs"]["O2_1t"]["sample_chunks"] == n  # small sample: the 1-thread leg keeps all of it
    bad = bytearray(want)
    bad[0] ^= 1
    assert bench.cpu_baseline(ctypes.addressof(buf), n, bytes(bad), min_s=0.01, reps=1)["digests_match_gpu"] is False


def _bench_module():
    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_bench_traffic_lookup_needs_the_same_build(tmp_path):
    """roofline.traffic is reported only from a PMC file measured on this very
    source id, kernel, variant and layout; a file from another build (e.g. a
    diagnostic build's suffixed id) yields null and says why."""
    import json
    bench = _bench_module()
    want = {"chunks": 131072, "pitch": 524288, "source_id": "abc", "kernel": "k_sha1_fixed", "variant": "310"}
    p = tmp_path / "traffic_r09.json"
    p.write_text(json.dumps({**want, "hbm_bytes_per_launch": 6.9e10}))
    assert bench.find_traffic(want, str(p)) == (6.9e10, f"{os.path.relpath(str(p), REPO)} (rocprofv3 --pmc, same source id)")
    t, note = bench.find_traffic({**want, "source_id": "abc-dbgbar"}, str(p))
    assert t is None and "another build" in note and "abc-dbgbar" in note
    # default: the committed traffic files; the newest one matching the product build wins
    files = sorted(f for f in os.listdir(os.path.join(REPO, "profiles")) if f.startswith("traffic_r"))
    newest = json.load(open(os.path.join(REPO, "profiles", files[-1])))
    mine = {k: newest[k] for k in want}
    t, note = bench.find_traffic(mine)
    assert t == newest["hbm_bytes_per_launch"] and files[-1] in note


def test_bench_process_age_is_wall_time_since_start():
    import time
    bench = _bench_module()
    a = bench.process_age_s()
    time.sleep(0.3)
    b = bench.process_age_s()
    assert 0 <= a < 600 and 0.2 <= b - a <= 2.0
