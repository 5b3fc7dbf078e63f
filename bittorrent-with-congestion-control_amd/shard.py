"""shard.py -- how a chunk batch is split over GPUs.

Chunks are independent (chunk.c:20-21 carries no state between chunks), so
the multi-GPU path is an embarrassingly parallel split with no data-path
collective:
  * weak scaling (bench.py, BASELINE config 4): every rank owns a fixed count
    of chunks, global indices [rank*C, (rank+1)*C), and generates / hashes
    them in its own HBM;
  * strong split of one image (bt_sha1_chunks_host_multi in the C library):
    device g of G takes [g*n//G, (g+1)*n//G) -- identical formula.
The only cross-rank traffic is a host-side gather of the 20-byte digests,
done over a CPU (gloo) group after the timed region.
"""


def weak_range(rank, chunks_per_rank):
    """Global chunk indices owned by `rank` under weak scaling."""
    lo = rank * chunks_per_rank
    return lo, lo + chunks_per_rank


def block_range(n, world, rank):
    """Contiguous block split of n chunks (same formula as the C library)."""
    return n * rank // world, n * (rank + 1) // world


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
    buf = torch.zeros(cap, dtype=torch.uint8)
    if local:
        buf[:len(local)] = torch.frombuffer(bytearray(local), dtype=torch.uint8)
    parts = [torch.zeros(cap, dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0, group=group)
    if rank != 0:
        return None
    return b"".join(bytes(p[:int(s.item())].numpy().tobytes()) for p, s in zip(parts, sizes))
