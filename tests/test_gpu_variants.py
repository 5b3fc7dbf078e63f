"""GPU: the experiments library (`make experiments`), i.e. the hot-kernel
variants measured and rejected, still bit-exact.

The product library carries one hot kernel (k_sha1_fixed, 3-slot ring of one
128-byte line, plain loads); `bt_sha1_set_variant` refuses everything else
there (tests/test_abi.py).  The rejected ring depths (2, 4), two-line slots,
non-temporal loads and the LDS-DMA-staged kernel (k_sha1_lds) live only in
build_variants/experiments/libbtsha1.so, which `bench.py --ring/--lines/--nt`
and tools/gpu_session.sh load through BT_SHA1_LIB.  A measurement is only
worth comparing if the variant computes sha.c's digests, so a child process
loads that build and runs each variant over:
  * BASELINE config 2: 4096 synthetic 512 KiB chunks vs the reference golden
    (tests/golden/synth4096.txt), every digest;
  * the fixed-layout edge cases (lengths 0..64 KiB+63, odd and padded
    pitches, partial last waves) vs the oracle;
  * 0 .. 2*2*NBUF+2 remaining blocks (the ring's line-count boundaries);
  * the fused verify epilogue with planted mismatches (util.c:311-313);
  * an image whose short last chunk rides in the same launch (chunk.c:20).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, PKG, REPO

pytestmark = pytest.mark.gpu
EXP_LIB = os.path.join(REPO, "build_variants", "experiments", "libbtsha1.so")
CHUNK = 512 * 1024
LDS = 10
VARIANTS = [(2, 1, 0), (3, 1, 0), (4, 1, 0), (2, 2, 0), (2, 1, 1), (3, 1, 1), (2, 2, 1), (LDS, 1, 0), (LDS, 1, 1)]
LAYOUTS = [(0, 16, 5), (1, 16, 3), (55, 64, 65), (56, 64, 64), (64, 64, 63), (100, 112, 129), (128, 128, 64),
           (192, 192, 65), (448, 448, 70), (4096 + 17, 4096 + 32, 130), (65536 + 63, 65536 + 64, 66),
           (3 * 128 * 5, 3 * 128 * 5, 200), (1000, 1003, 67), (CHUNK, CHUNK + 256, 65)]


def _child():
    import torch
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, PKG)
    import btsha1 as bt
    import py_oracle as orc

    assert torch.cuda.is_available()
    assert os.path.samefile(bt.LIB_PATH, EXP_LIB), bt.LIB_PATH
    assert bt.source_id().endswith("-exp"), bt.source_id()
    bt.set_latency_batch(0)  # every fixed-layout batch takes the selected hot-kernel variant
    bt.set_chain_batch(0)
    results = []

    def dev(data):
        t = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
        if data:
            t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        return t

    def digests(t, n):
        raw = bytes(t[:20 * n].cpu().numpy().tobytes())
        return [raw[20 * i:20 * i + 20] for i in range(n)]

    golden = [bytes.fromhex(l.split()[1]) for l in open(os.path.join(GOLDEN, "synth4096.txt"))
              if l.strip() and not l.startswith("#")]
    synth = torch.empty(4096 * CHUNK, dtype=torch.uint8, device="cuda")
    bt.fill_synthetic(synth.data_ptr(), 4096 * CHUNK, 0, orc.SEED_SYNTH)
    torch.cuda.synchronize()

    for v in VARIANTS:
        bt.set_variant(*v)
        name = f"{v[0]}x{v[1]}{' nt' if v[2] else ''}"
        kernel = "k_sha1_lds" if v[0] == LDS else "k_sha1_fixed"
        assert bt.kernel_name(4096) == kernel, (v, bt.kernel_name(4096))

        # config 2, every digest against the reference golden
        out = torch.zeros(20 * 4096, dtype=torch.uint8, device="cuda")
        bt.chunks_dev(synth.data_ptr(), 4096, CHUNK, CHUNK, out.data_ptr())
        torch.cuda.synchronize()
        results.append({"variant": name, "case": "config2 4096", "ok": digests(out, 4096) == golden})

        # fused verify: 1000 chunks, four planted mismatches
        n, bad = 1000, {0, 17, 511, 999}
        exp = bytearray(b"".join(golden[:n]))
        for i in bad:
            exp[20 * i + (i % 20)] ^= 1
        ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        d_exp = dev(bytes(exp))
        bt.verify_dev(synth.data_ptr(), n, CHUNK, CHUNK, d_exp.data_ptr(), ok.data_ptr(), None)
        torch.cuda.synchronize()
        flags = ok.cpu().tolist()
        results.append({"variant": name, "case": "verify",
                        "ok": flags == [0 if i in bad else 1 for i in range(n)]})

        # fixed layouts vs the oracle
        good = True
        for length, pitch, n in LAYOUTS:
            host = bytes(orc.fill_synthetic(pitch * (n - 1) + length, 11, 0xC0FFEE))
            d = dev(host)
            out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
            bt.chunks_dev(d.data_ptr(), n, length, pitch, out.data_ptr())
            torch.cuda.synchronize()
            good = good and digests(out, n) == [orc.sha1(host[i * pitch:i * pitch + length]) for i in range(n)]
        results.append({"variant": name, "case": "layouts", "ok": good})

        # remaining blocks 0 .. 2*2*NBUF+2 after the ring's last full slot
        deepest = 4 if v[0] == LDS else v[0] * v[1]
        good = True
        for blocks in range(0, 2 * 2 * deepest + 3):
            for r in (0, 5, 56):
                length = 64 * blocks + r
                n = 70
                pitch = (length + 15) // 16 * 16 or 16
                host = bytes(orc.fill_synthetic(pitch * n, blocks, deepest))
                d = dev(host)
                out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
                bt.chunks_dev(d.data_ptr(), n, length, pitch, out.data_ptr())
                torch.cuda.synchronize()
                got = digests(out, n)
                good = good and all(got[i] == orc.sha1(host[i * pitch:i * pitch + length]) for i in (0, 1, 63, 64, 69))
        results.append({"variant": name, "case": "line counts", "ok": good})

        # image + short tail in the same launch (the LDS variant hands the tail to the ragged kernel)
        good = True
        for chunk_len in (4096, 64 * 1024):
            for nfull in (0, 1, 64, 65, 130):
                for rem in (1, 55, 56, 64, 1000, chunk_len - 1):
                    img = bytes(orc.fill_synthetic(nfull * chunk_len + rem, nfull + rem, 0x7A11))
                    good = good and bt.chunks_host(img, chunk_len=chunk_len) == orc.hash_chunks(img, chunk_len)
        results.append({"variant": name, "case": "image tail", "ok": good})
    bt.set_variant(3, 1, 0)
    print("VARIANT_RESULTS " + json.dumps(results), flush=True)


def test_rejected_variants_bit_exact_in_the_experiments_build():
    assert os.path.exists(EXP_LIB), "build_variants/experiments/libbtsha1.so missing: run `make experiments` first"
    env = dict(os.environ, BT_SHA1_LIB=EXP_LIB, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "child"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("VARIANT_RESULTS ")]
    assert len(line) == 1, r.stdout[-2000:]
    results = json.loads(line[0].split(" ", 1)[1])
    assert len(results) == 5 * len(VARIANTS)
    bad = [c for c in results if not c["ok"]]
    assert not bad, bad


if __name__ == "__main__" and sys.argv[1:] == ["child"]:
    _child()
