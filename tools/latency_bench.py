#!/usr/bin/env python3
"""tools/latency_bench.py -- latency of the single-message and ragged paths.

The hot kernel is throughput-shaped (131072 chunks in flight).  The drop-in
callers that keep the reference's synchronous contract pay a chunk's serial
chain instead: util.c:311 calls shahash once per received chunk, and
make_chunks hashes its short last chunk alone (chunk.c:20-21).  This prints
one JSON line per measurement (median of --reps):

  shahash_512k      shahash() of one 512 KiB host buffer, call to return
  shahash_<n>B      shahash() of a short message: the fixed cost of a drop-in call
  ragged_1x512k     bt_sha1_ragged_dev over one device-resident 512 KiB message
  ragged_1x512k_u   the same message at an odd byte offset (unaligned loads)
  ragged_4096       4096 device-resident messages of 480-544 KiB at 16-byte
                    aligned offsets (GiB/s of message bytes)
  ragged_4096_u     the same lengths at arbitrary byte offsets
  update_1484       SHA1Update of one 512 KiB chunk fed as 1484-byte payloads
                    (save_data_packet's granule, util.c:275) + SHA1Final
  batch_<n>_<mode>  n device-resident 512 KiB chunks through the hot kernel
                    (fixed) or the two-wave latency kernel (lat), kernel time
  verifier_b1       bt_sha1_verifier with batch 1: submit -> verdict
Digests are checked against the oracle (hashlib is not used).
"""
import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "bittorrent-with-congestion-control_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

CHUNK = 512 * 1024


def emit(name, samples_s, extra=None):
    med = statistics.median(samples_s)
    d = {"case": name, "median_ms": round(med * 1e3, 4), "min_ms": round(min(samples_s) * 1e3, 4),
         "reps": len(samples_s)}
    d.update(extra or {})
    print(json.dumps(d), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    args = ap.parse_args()
    import numpy as np
    import torch
    import btsha1 as bt
    import py_oracle as orc

    rng = np.random.default_rng(7)
    msg = bytes(orc.fill_synthetic(CHUNK, 0, orc.SEED_SYNTH))
    want = orc.sha1(msg)

    # shahash: host buffer in, 20 bytes out, synchronous (chunk.c:33-49).
    assert bt.shahash(msg) == want
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        got = bt.shahash(msg)
        ts.append(time.perf_counter() - t0)
    assert got == want
    emit("shahash_512k", ts)
    # Fixed cost of one drop-in call: short messages (one launch of the chain
    # kernel on pinned host memory + the spin on its completion word).
    for ln in (0, 55, 1484, 16384):
        m = msg[:ln]
        assert bt.shahash(m) == orc.sha1(m)
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            bt.shahash(m)
            ts.append(time.perf_counter() - t0)
        emit(f"shahash_{ln}B", ts)

    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    dev = torch.empty(CHUNK + 4096, dtype=torch.uint8, device="cuda")
    out = torch.zeros(20 * 4096, dtype=torch.uint8, device="cuda")

    def ragged(base, offs, lens):
        o = torch.tensor(offs, dtype=torch.int64, device="cuda")
        ln = torch.tensor(lens, dtype=torch.int32, device="cuda")
        res = []
        for _ in range(args.reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            bt.ragged_dev(base, o.data_ptr(), ln.data_ptr(), len(offs), out.data_ptr(), s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            res.append(a.elapsed_time(b) * 1e-3)
        return res[1:]

    prev_chain = bt.set_chain_batch(0)
    for kname, thr in (("k_sha1_ragged", 0), ("k_sha1_chain", 1 << 62)):
        bt.set_chain_batch(thr)
        for name, off in (("ragged_1x512k", 0), ("ragged_1x512k_u", 3)):
            dev[off:off + CHUNK].copy_(torch.frombuffer(bytearray(msg), dtype=torch.uint8))
            ts = ragged(dev.data_ptr(), [off], [CHUNK])
            assert bytes(out[:20].cpu().numpy().tobytes()) == want, name
            emit(name + ("_chain" if thr else ""), ts, {"kernel": kname})
    bt.set_chain_batch(0)

    n = 4096
    lens = [int(x) for x in rng.integers(480 * 1024, 544 * 1024, n)]
    prev_lat = bt.set_latency_batch(2**64 - 1)
    for name, aligned, lat in (("ragged_4096", True, 0), ("ragged_4096_u", False, 0),
                               ("ragged_4096_latr", True, 2**64 - 1), ("ragged_4096_u_latr", False, 2**64 - 1)):
        bt.set_latency_batch(lat)
        offs, pos = [], 0
        for ln in lens:
            pos += int(rng.integers(0, 16)) if not aligned else 0
            offs.append(pos)
            pos += ln
            pos = (pos + 15) & ~15 if aligned else pos
        total = pos + 64
        big = torch.empty(total, dtype=torch.uint8, device="cuda")
        bt.fill_synthetic(big.data_ptr(), total, 12345, orc.SEED_SYNTH, s.cuda_stream)
        torch.cuda.synchronize()
        ts = ragged(big.data_ptr(), offs, lens)
        host = big.cpu().numpy()
        for i in list(range(0, n, 511)) + [n - 1]:
            assert bytes(out[20 * i:20 * i + 20].cpu().numpy().tobytes()) == \
                orc.sha1(host[offs[i]:offs[i] + lens[i]].tobytes()), (name, i)
        med = statistics.median(ts)
        emit(name, ts, {"kernel": "k_sha1_lat_ragged" if lat else "k_sha1_ragged", "messages": n,
                        "GiB_per_s": round(sum(lens) / med / 2**30, 2)})
        del big
    bt.set_latency_batch(prev_lat)

    # Streaming API at the peer's packet granule.
    ts = []
    for _ in range(max(1, args.reps // 3)):
        t0 = time.perf_counter()
        h = bt.Sha1()
        for o in range(0, CHUNK, 1484):
            h.update(msg[o:o + 1484])
        got = h.final()
        ts.append(time.perf_counter() - t0)
    assert got == want
    emit("update_1484", ts)

    # Device-resident batches of n 512 KiB chunks: the two-wave latency kernel
    # (k_sha1_lat) against the hot kernel (k_sha1_fixed), kernel time only.
    nmax = 65536
    big = torch.empty(nmax * CHUNK, dtype=torch.uint8, device="cuda")
    bt.fill_synthetic(big.data_ptr(), nmax * CHUNK, 0, orc.SEED_SYNTH, s.cuda_stream)
    dig = torch.zeros(20 * nmax, dtype=torch.uint8, device="cuda")
    golden = {}
    gpath = os.path.join(REPO, "tests", "golden", "synth4096.txt")
    for line in open(gpath):
        if not line.startswith("#"):
            i, h = line.split()
            golden[int(i)] = h
    prev = bt.set_latency_batch(0)
    prev_chain_fixed = bt.set_chain_batch(0)
    for n in (1, 64, 256, 512, 1024, 2048, 4096, 16384, 24576, 32768, 65536):
        for mode, thr, cthr in (("fixed", 0, 0), ("lat", 1 << 62, 0), ("chainfixed", 1 << 62, 1 << 62)):
            if mode == "chainfixed" and n > 4096:
                continue
            bt.set_latency_batch(thr)
            bt.set_chain_batch(cthr)
            res = []
            for _ in range(max(3, args.reps // 2) + 1):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                bt.chunks_dev(big.data_ptr(), n, CHUNK, CHUNK, dig.data_ptr(), s.cuda_stream)
                b.record(s)
                torch.cuda.synchronize()
                res.append(a.elapsed_time(b) * 1e-3)
            raw = dig[:20 * min(n, 4096)].cpu().numpy().tobytes()
            assert all(raw[20 * i:20 * i + 20].hex() == golden[i] for i in range(min(n, 4096))), (mode, n)
            med = statistics.median(res[1:])
            emit(f"batch_{n}_{mode}", res[1:], {"chunks": n, "GiB_per_s": round(n * CHUNK / med / 2**30, 2)})
    bt.set_latency_batch(prev)
    bt.set_chain_batch(prev_chain_fixed)
    # The same chunks as ragged messages through the chain kernel (one
    # two-wave workgroup per chunk).
    bt.set_chain_batch(1 << 62)
    for n in (1, 64, 256):
        o = torch.arange(n, dtype=torch.int64, device="cuda") * CHUNK
        ln = torch.full((n,), CHUNK, dtype=torch.int32, device="cuda")
        res = []
        for _ in range(max(3, args.reps // 2) + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            bt.ragged_dev(big.data_ptr(), o.data_ptr(), ln.data_ptr(), n, dig.data_ptr(), s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            res.append(a.elapsed_time(b) * 1e-3)
        raw = dig[:20 * n].cpu().numpy().tobytes()
        assert all(raw[20 * i:20 * i + 20].hex() == golden[i] for i in range(n)), ("chain", n)
        med = statistics.median(res[1:])
        emit(f"batch_{n}_chain", res[1:], {"chunks": n, "GiB_per_s": round(n * CHUNK / med / 2**30, 2)})
    bt.set_chain_batch(prev_chain)
    del big

    v = bt.Verifier(batch=1, nstreams=2)
    ts = []
    for i in range(args.reps):
        t0 = time.perf_counter()
        v.submit(msg, want, tag=i)
        r = v.drain()
        ts.append(time.perf_counter() - t0)
        assert r == [(i, True, want)], r
    v.close()
    emit("verifier_b1", ts)


if __name__ == "__main__":
    main()
