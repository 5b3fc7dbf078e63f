"""shard.py -- how a chunk batch is split over GPUs, and the
rank logic bench.py runs on every rank.

Chunks are independent (chunk.c:20-21 carries no state between chunks), so
the multi-GPU path is an embarrassingly parallel split with no data-path
collective:
  * weak scaling (bench.py, BASELINE config 4): every rank owns a fixed count
    of chunks, global indices [rank*C, (rank+1)*C), and generates / hashes
    them in its own HBM;
  * strong split of one image (bt_sha1_chunks_host_devices in the C library):
    worker g of G takes [g*n//G, (g+1)*n//G) -- identical formula.
Ranks meet only on a CPU (gloo) group: the timing barriers, the
max-over-ranks reduction of the wall times, and a host-side gather of the
20-byte digests after the timed region.  No RCCL collective is involved.
"""
import time


def weak_range(rank, chunks_per_rank):
    """Global chunk indices owned by `rank` under weak scaling."""
    lo = rank * chunks_per_rank
    return lo, lo + chunks_per_rank


def block_range(n, world, rank):
    """Contiguous block split of n chunks (same formula as the C library)."""
    return n * rank // world, n * (rank + 1) // world


def sample_chunks(world, chunks_per_rank, k):
    """(rank, global chunk index) of k chunks of every rank under weak scaling:
    the rank's first and last chunk and k-2 evenly between (bench.py's
    `digest_sample`, checked against the oracle by the tests)."""
    out = []
    for r in range(world):
        lo, hi = weak_range(r, chunks_per_rank)
        picks = sorted({lo + (hi - 1 - lo) * j // max(1, k - 1) for j in range(k)}) if hi > lo and k > 0 else []
        out += [(r, g) for g in picks]
    return out


def barrier(world, group=None):
    if world > 1:
        import torch.distributed as dist
        dist.barrier(group=group)


def gather_floats(values, world, group=None):
    """Every rank's list of floats, in rank order (all ranks get all)."""
    if world == 1:
        return [list(values)]
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return [[float(x) for x in p] for p in parts]


def gather_objects(obj, world, group=None):
    """Every rank's (picklable, small) object, in rank order, on every rank."""
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj, group=group)
    return out


def _bdf(addr, with_function=True):
    """A PCI address in one spelling: lowercase, 4-digit domain; without the
    function number when with_function is False."""
    if not addr:
        return None
    a = str(addr).strip().lower()
    if a.count(":") == 1:  # bus:device.function without a domain
        a = "0000:" + a
    dom, bus, rest = a.split(":", 2)
    dev, _, fn = rest.partition(".")
    out = f"{int(dom, 16):04x}:{int(bus, 16):02x}:{int(dev, 16):02x}"
    return f"{out}.{int(fn or '0', 16)}" if with_function else out


def device_keys(idents):
    """One key per rank naming the physical GPU it drove: (host, PCI address,
    UUID), every rank's key built the same way, so one GPU can never get two
    keys because two ranks read it through different sources:
      * the address is amdsmi's full domain:bus:device.function (`smi_bdf`)
        when EVERY rank has it -- partitions of one GPU differ only in the
        function number -- else HIP's domain:bus:device for every rank
        (`pci_bdf` without its fixed .0: the coarser key, so two partitions
        then count as one GPU rather than one GPU as two);
      * the UUID only when every rank got it from the same source (amdsmi
        and HIP spell one GPU's UUID differently), else none;
      * the host keeps two nodes' equal PCI addresses apart (multi-node)."""
    full = bool(idents) and all(i.get("smi_bdf") for i in idents)
    sources = {i.get("uuid_source") for i in idents}
    same_uuid = len(sources) == 1 and None not in sources
    keys = []
    for i in idents:
        addr = _bdf(i.get("smi_bdf")) if full else _bdf(i.get("pci_bdf"), with_function=False)
        keys.append((i.get("host"), addr, i.get("uuid") if same_uuid else None))
    return keys


def distinct_devices(idents):
    """How many distinct GPUs the ranks drove (bench.py's `distinct_gpus`)."""
    return len(set(device_keys(idents)))


def check_distinct_devices(idents, world, allow_shared=False):
    """An N-GPU line must come from N distinct GPUs.  `idents` is every rank's
    {"rank", "host", "pci_bdf", "uuid", ...}.  Returns a message (every rank
    then exits before the timed region) when fewer than `world` distinct GPUs
    drive the ranks -- whatever each rank's device_count says: one device
    visible per rank (*_VISIBLE_DEVICES) is fine as long as the devices
    differ -- or when the gather is incomplete; None when the launch is sound.
    allow_shared (bench.py --rehearse-shared-gpu, recorded in the line) lets
    ranks share GPUs on purpose: the rank path rehearsed on one GPU."""
    if world <= 1:
        return None
    if len(idents) != world:
        return f"identity gather returned {len(idents)} of {world} ranks"
    if allow_shared:
        return None
    seen = {}
    for i, key in zip(idents, device_keys(idents)):
        seen.setdefault(key, []).append(i.get("rank"))
    if len(seen) == world:
        return None
    dup = {k: ranks for k, ranks in seen.items() if len(ranks) > 1}
    return (f"{world} ranks but {len(seen)} distinct GPU(s): ranks share a GPU ("
            + ", ".join(f"{k[1]} on {k[0]} <- ranks {ranks}" for k, ranks in sorted(dup.items(), key=str))
            + "); pass --rehearse-shared-gpu to run the rank path on shared GPUs on purpose")


def gather_digests(local: bytes, world, rank, group=None):
    """Host-side gather of per-rank digest slices to rank 0, in rank order
    (== global chunk order for both splits above).  Returns the concatenation
    on rank 0 and None elsewhere.  Slices may differ in length."""
    if world == 1:
        return local
    import torch
    import torch.distributed as dist
    n = torch.tensor([len(local)], dtype=torch.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    cap = int(max(s.item() for s in sizes))
    buf = torch.zeros(max(cap, 1), dtype=torch.uint8)
    if local:
        buf[:len(local)] = torch.frombuffer(bytearray(local), dtype=torch.uint8)
    parts = [torch.zeros(max(cap, 1), dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0, group=group)
    if rank != 0:
        return None
    return b"".join(bytes(p[:int(s.item())].numpy().tobytes()) for p, s in zip(parts, sizes))


def run_rank(hasher, steps, warmup, world, rank, group=None):
    """The per-rank benchmark protocol of bench.py (the driver's contract):
    `warmup` untimed steps; barrier + sync; `steps` timed steps; sync +
    barrier; then the max over ranks of the wall time and of the hot kernel's
    average time, and the digests gathered to rank 0 in global chunk order.

    `hasher` provides step(i) (launch one pass over the rank's chunks),
    sync() (wait for the device), kernel_ms() (the hot kernel's average launch
    time over the timed steps, or None) and digests() (the rank's digests,
    bytes).  bench.py passes the HIP hasher; tests pass a CPU stub.
    Returns a dict on every rank ('digests' only on rank 0)."""
    for i in range(warmup):
        hasher.step(-1 - i)
    hasher.sync()
    barrier(world, group)
    hasher.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        hasher.step(i)
    hasher.sync()
    barrier(world, group)
    wall = time.perf_counter() - t0
    kern = hasher.kernel_ms()
    per_rank = gather_floats([wall, -1.0 if kern is None else kern], world, group)
    digests = gather_digests(hasher.digests(), world, rank, group)
    return {
        "wall_max": max(w for w, _ in per_rank),
        "kernel_ms_max": max(k for _, k in per_rank) if kern is not None else None,
        "per_rank": per_rank,
        "digests": digests,
    }
