"""GPU: the barrier-accounting build (`make dbgbar`) on the shapes that stress
the latency kernels' barrier counts.

k_sha1_lat, k_sha1_chain and k_sha1_lat_ragged split each chain between a
loader/schedule wave S and a round wave R that meet at s_barrier from
DIFFERENT call sites; s_barrier counts waves, so the kernels are correct only
while both waves execute exactly the count the invariant in sha1_kernels.hip
("Barrier accounting") predicts -- and that count derives from the padding
block count of sha.c:536-543 (one padding block, or two when the tail holds
r >= 56 bytes).  The -DBT_SHA1_DEBUG_BARRIERS build counts each wave's
barriers and tallies {waves checked, barriers executed, misses}.

The child process loads that build (BT_SHA1_LIB) and runs, each pinned to its
kernel: tails with r >= 56 and r < 56, the chain kernel at 63/64/65 and
128/129 blocks (its 64-block loader batches), the streaming API's midstate
launches, the 2- and 3-slot forms of k_sha1_lat (1 and > 1 workgroups per CU)
incl. the fused verify and an image tail, and ragged batches whose longest
message sits in the LAST lane of its workgroup.  For every case it checks
the digests against the oracle, zero misses, and the EXACT wave and barrier
totals computed here from the invariant -- so the tallies prove the counting
build is what ran, and which kernel (S/R pairs per workgroup) ran.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu
DBG_LIB = os.path.join(REPO, "build_variants", "dbgbar", "libbtsha1.so")


def nb_total(length):
    """Blocks of one message incl. MD padding (sha.c:536-543)."""
    return (length >> 6) + (2 if (length & 63) >= 56 else 1)


def _child():
    import torch
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, PKG)
    import btsha1 as bt
    import py_oracle as orc

    assert torch.cuda.is_available()
    assert os.path.samefile(bt.LIB_PATH, DBG_LIB), bt.LIB_PATH
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    bt.debug_barrier_stats(reset=True)
    results = []

    def pin(chain, lat):
        bt.set_chain_batch(1 << 62 if chain else 0)
        bt.set_latency_batch(1 << 62 if lat else 0)

    def record(name, want, ok):
        got = bt.debug_barrier_stats(reset=True)
        results.append({"case": name, "want": list(want), "got": list(got), "digests_ok": bool(ok)})

    def dev(data):
        t = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
        if data:
            t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        return t

    def fixed(name, n, length, pitch, kernel, seed, verify=False):
        data = bytes(orc.fill_synthetic(n * pitch, seed, 0xBA77))
        d = dev(data)
        out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
        assert bt.kernel_name(n) == kernel, (name, bt.kernel_name(n))
        want_dig = b"".join(orc.sha1(data[i * pitch:i * pitch + length]) for i in range(n))
        if verify:
            exp = bytearray(want_dig)
            for i in range(0, n, 7):
                exp[20 * i] ^= 1  # every 7th chunk must fail util.c:313's compare
            e = dev(bytes(exp))
            ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
            bt.verify_dev(d.data_ptr(), n, length, pitch, e.data_ptr(), ok.data_ptr(), out.data_ptr())
            torch.cuda.synchronize()
            good = [int(x) for x in ok.cpu()] == [0 if i % 7 == 0 else 1 for i in range(n)]
        else:
            bt.chunks_dev(d.data_ptr(), n, length, pitch, out.data_ptr())
            torch.cuda.synchronize()
            good = True
        good = good and bytes(out.cpu().numpy().tobytes()) == want_dig
        if kernel == "k_sha1_chain":
            per = 2 * ((nb_total(length) + 63) // 64 + 1)
            want = (2 * n, n * per)
        else:
            grid = (n + 63) // 64
            slots = 3 if grid > cus else 2
            want = (2 * grid, 2 * grid * (nb_total(length) + slots - 1))
        record(name, want, good)

    # ---- k_sha1_chain: one two-wave workgroup per message, 64-block batches
    pin(chain=True, lat=True)
    for k, length in enumerate([62 * 64, 63 * 64, 64 * 64, 61 * 64 + 60, 62 * 64 + 56, 63 * 64 + 57,
                                127 * 64, 127 * 64 + 60, 55, 56, 0]):
        pitch = (length + 15) // 16 * 16 or 16
        fixed(f"chain len={length} nb={nb_total(length)}", 3, length, pitch, "k_sha1_chain", 100 + k)
    fixed("chain verify", 5, 64 * 64, 64 * 64, "k_sha1_chain", 120, verify=True)
    # image with a short last chunk (the make_chunks tail rides in the same launch)
    img = bytes(orc.fill_synthetic(5 * 4096 + 4000, 130, 0xBA77))
    got = bt.chunks_host(img, 4096)
    want_dig = [orc.sha1(img[i:i + 4096]) for i in range(0, len(img), 4096)]
    record("chain image + tail", (2 * 6, 5 * 2 * ((nb_total(4096) + 63) // 64 + 1) + 2 * ((nb_total(4000) + 63) // 64 + 1)),
           got == want_dig)
    # drop-ins: shahash (chain kernel) and the SHA1Update / SHA1Final midstates
    for length in (63 * 64 + 60, 64 * 64 + 56):
        msg = bytes(orc.fill_synthetic(length, 140 + length, 0xBA77))
        ok = bt.shahash(msg) == orc.sha1(msg)
        record(f"shahash len={length}", (2, 2 * ((nb_total(length) + 63) // 64 + 1)), ok)
    for nb in (63, 64, 65, 129):
        msg = bytes(orc.fill_synthetic(64 * nb, 150 + nb, 0xBA77))
        ok = bt.Sha1().update(msg).final() == orc.sha1(msg)
        # update: one midstate launch of nb blocks; final: one padding block
        record(f"SHA1Update {nb} blocks + SHA1Final", (4, 2 * ((nb + 63) // 64 + 1) + 2 * 2), ok)

    # ---- k_sha1_lat: 64 chunks per two-wave workgroup
    pin(chain=False, lat=True)
    fixed("lat 2-slot r=56", 100, 4096 + 56, 4160, "k_sha1_lat", 200)
    fixed("lat 2-slot r=40", 130, 1000, 1008, "k_sha1_lat", 201)
    fixed("lat 2-slot r=0 verify", 100, 4096, 4096, "k_sha1_lat", 202, verify=True)
    fixed("lat 3-slot r=60", 64 * cus + 64, 1024 + 60, 1088, "k_sha1_lat", 203)
    fixed("lat 3-slot odd count r=63", 64 * cus + 1, 64 * 3 + 63, 256, "k_sha1_lat", 204)
    img = bytes(orc.fill_synthetic(100 * 1024 + 1020, 205, 0xBA77))
    got = bt.chunks_host(img, 1024)
    want_dig = [orc.sha1(img[i:i + 1024]) for i in range(0, len(img), 1024)]
    record("lat image + tail r=60", (6, 2 * 2 * (nb_total(1024) + 1) + 2 * (nb_total(1020) + 1)), got == want_dig)

    # ---- k_sha1_lat_ragged: the wave runs to its longest message; put it in lane 63
    pin(chain=False, lat=True)
    for name, n, seed in (("lat_ragged 2-slot", 600, 300), ("lat_ragged 3-slot", 64 * cus + 100, 301)):
        import random
        rng = random.Random(seed)
        lens = [rng.randrange(0, 1500) for _ in range(n)]
        for g in range(0, n, 64):
            last = min(g + 63, n - 1)
            lens[last] = 1600 + 60 if (g // 64) % 2 else 1600 + 20  # longest, r >= 56 on every other group
        blob, offs = bytearray(), []
        for i, ln in enumerate(lens):
            blob += bytes(i % 5)  # odd alignments
            offs.append(len(blob))
            blob += bytes(orc.fill_synthetic(ln, 1000 * i, seed))
        d = dev(bytes(blob))
        o = torch.tensor(offs, dtype=torch.int64, device="cuda")
        ln_t = torch.tensor(lens, dtype=torch.int32, device="cuda")
        out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
        bt.ragged_dev(d.data_ptr(), o.data_ptr(), ln_t.data_ptr(), n, out.data_ptr())
        torch.cuda.synchronize()
        good = bytes(out.cpu().numpy().tobytes()) == b"".join(
            orc.sha1(bytes(blob[offs[i]:offs[i] + lens[i]])) for i in range(n))
        grid = (n + 63) // 64
        slots = 3 if grid > cus else 2
        bars = 0
        for g in range(grid):
            idx = [min(g * 64 + j, n - 1) for j in range(64)]  # lanes past n re-hash message n-1
            bars += 2 * (max(nb_total(lens[i]) for i in idx) + slots - 1)
        record(name, (2 * grid, bars), good)
    print("BARRIER_RESULTS " + json.dumps(results), flush=True)


def test_barrier_accounting_build_matches_invariant():
    assert os.path.exists(DBG_LIB), "build_variants/dbgbar/libbtsha1.so missing: run `make dbgbar` first"
    env = dict(os.environ, BT_SHA1_LIB=DBG_LIB, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "child"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("BARRIER_RESULTS ")]
    assert len(line) == 1, r.stdout[-2000:]
    results = json.loads(line[0].split(" ", 1)[1])
    assert len(results) == 27
    bad = [c for c in results if not c["digests_ok"] or c["got"][2] != 0 or c["got"][:2] != c["want"]]
    assert not bad, bad


if __name__ == "__main__" and sys.argv[1:] == ["child"]:
    _child()
