"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
reference's golden vectors.  Bit-exact everywhere (integer/byte work)."""
import contextlib
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys
import threading
import time

import pytest

from conftest import GOLDEN, PKG, REPO, c_tar_bytes, load_btsha1, read_pairs

pytestmark = pytest.mark.gpu
CHUNK = 512 * 1024


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "gpu tests need a HIP device"
    return t


@pytest.fixture(scope="module")
def bt(torch):
    m = load_btsha1()
    assert m.device_count() >= 1
    return m


def to_dev(torch, data: bytes, pad=0):
    t = torch.zeros(len(data) + pad + 16, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t


def digests_of(torch, t, n):
    return [bytes(t[20 * i:20 * i + 20].cpu().numpy().tobytes()) for i in range(n)]


def kat_data():
    return {"abc": b"abc", "dash": b"dash", "empty": b"",
            "nist448": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
            "zeros_512k": bytes(CHUNK), "ff_512k": b"\xff" * CHUNK,
            "iota_512k": bytes(i & 255 for i in range(CHUNK)), "million_a": b"a" * 1000000}


def test_shahash_kats(bt):
    data = kat_data()
    for name, n, h in read_pairs("kat.txt"):
        assert bt.shahash(data[name]).hex() == h, name
        # chunk.c:48: nothing of the message or the state is left behind
        assert bt.debug_dropin_residue(0) == 0, name


def test_dropin_calls_leave_no_staged_message_behind(bt, oracle):
    """The reference's wipe contract (chunk.c:48 zeroes shahash's context;
    sha.c:165-174, 526 burn SHA1Update's stack): after every drop-in call the
    pinned staging that held the caller's message and the chaining state reads
    all zero -- a 512 KiB chunk of nonzero bytes through shahash, and a
    streaming SHA1Update / SHA1Final sequence -- and the digests are still
    bit-exact."""
    chunk = bytes(oracle.fill_synthetic(512 * 1024, 99, 0x51A7))
    assert chunk.count(0) < len(chunk) // 100
    assert bt.shahash(chunk) == oracle.sha1(chunk)
    assert bt.debug_dropin_residue(0) == 0
    s = bt.Sha1()
    for a, b in ((0, 100), (100, 64 * 1000 + 7), (64 * 1000 + 7, len(chunk))):
        s.update(chunk[a:b])
        assert bt.debug_dropin_residue(0) == 0, (a, b)
    assert s.final() == oracle.sha1(chunk)
    assert bt.debug_dropin_residue(0) == 0
    with pytest.raises(bt.BtSha1Error):
        bt.debug_dropin_residue(-1)


def test_shahash_either_side_of_the_hot_kernel_limit(bt, oracle):
    """shahash runs the chain kernel on the pinned staging copy: messages on
    both sides of the hot kernel's 32-bit offset limit (~64 MiB, where the
    fixed-layout paths switch kernels), plus short messages at every residue
    mod 64 (one or two padding blocks built by the loader wave)."""
    limit = ((1 << 32) - 4096) // 64  # largest 16-byte pitch the hot kernel takes
    for n in (limit - 16 - 7, limit + 1):
        msg = bytes(oracle.fill_synthetic(n, n, 0x51A7))
        assert bt.shahash(msg) == oracle.sha1(msg), n
    base = bytes(oracle.fill_synthetic(200, 1, 0x51A7))
    for n in range(0, 200):
        assert bt.shahash(base[:n]) == oracle.sha1(base[:n]), n


def test_streaming_api_kats_random_splits(bt):
    data = kat_data()
    rng = random.Random(1)
    for name, n, h in read_pairs("kat.txt"):
        d = data[name]
        s = bt.Sha1()
        i = 0
        while i < len(d):
            j = min(len(d), i + rng.choice([1, 3, 63, 64, 65, 640, 4096, 100000]))
            s.update(d[i:j])
            i = j
        assert s.final().hex() == h, name


def test_streaming_context_fields(bt, oracle):
    s = bt.Sha1().update(b"x" * 100)
    assert s.ctx.totalLength == 800 and s.ctx.bufferLength == 36
    assert list(s.ctx.hash) == oracle.compress_blocks(
        [0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476, 0xc3d2e1f0], b"x" * 64)


@contextlib.contextmanager
def ragged_mode(bt, mode):
    """Pin ragged batches to the chain kernel ("chain": one workgroup per
    message), the ragged latency kernel ("latr": loader / round waves per 64
    messages) or the one-message-per-lane ragged kernel ("lanes")."""
    prev = bt.set_chain_batch(1 << 62 if mode == "chain" else 0)
    prev_lat = bt.set_latency_batch(0 if mode == "lanes" else 1 << 62)
    try:
        yield
    finally:
        bt.set_chain_batch(prev)
        bt.set_latency_batch(prev_lat)


@pytest.fixture(params=["chain", "latr", "lanes"])
def rmode(bt, request):
    with ragged_mode(bt, request.param):
        yield request.param


def test_edge_lengths_ragged_kernel(bt, torch, oracle, rmode):
    rows = read_pairs("edge_lengths.txt")
    stream = bytes(oracle.fill_synthetic(max(int(n) for n, _ in rows), 0, oracle.SEED_EDGE))
    d = to_dev(torch, stream)
    n = len(rows)
    offs = torch.zeros(n, dtype=torch.int64, device="cuda")
    lens = torch.tensor([int(x) for x, _ in rows], dtype=torch.int32, device="cuda")
    out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
    bt.ragged_dev(d.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, out.data_ptr())
    torch.cuda.synchronize()
    assert [x.hex() for x in digests_of(torch, out, n)] == [h for _, h in rows]


def test_ragged_golden_batch_unaligned(bt, torch, oracle, rmode):
    rows = read_pairs("ragged.txt")
    msgs = [bytes(oracle.fill_synthetic(int(n), int(k) * 1024, oracle.SEED_RAGGED)) for k, n, _ in rows]
    # pack with deliberately odd offsets (1..7 bytes of slack) to hit every alignment
    blob, offs = bytearray(), []
    for i, m in enumerate(msgs):
        blob += bytes(1 + i % 7)
        offs.append(len(blob))
        blob += m
    d = to_dev(torch, bytes(blob))
    o = torch.tensor(offs, dtype=torch.int64, device="cuda")
    l = torch.tensor([len(m) for m in msgs], dtype=torch.int32, device="cuda")
    out = torch.zeros(20 * len(msgs), dtype=torch.uint8, device="cuda")
    bt.ragged_dev(d.data_ptr(), o.data_ptr(), l.data_ptr(), len(msgs), out.data_ptr())
    torch.cuda.synchronize()
    assert [x.hex() for x in digests_of(torch, out, len(msgs))] == [h for _, _, h in rows]


def test_device_generator_matches_oracle(bt, torch, oracle):
    for nbytes, first in [(CHUNK, 7 * 65536), (1000, 3), (4096 + 8, 2**40 + 1)]:
        t = torch.zeros(nbytes + 32, dtype=torch.uint8, device="cuda")
        bt.fill_synthetic(t.data_ptr(), nbytes, first, oracle.SEED_SYNTH)
        torch.cuda.synchronize()
        assert bytes(t[:nbytes].cpu().numpy().tobytes()) == bytes(oracle.fill_synthetic(nbytes, first, oracle.SEED_SYNTH))
        assert int(t[nbytes:].sum()) == 0  # no overrun


@pytest.fixture(scope="module")
def synth4096(bt, torch, oracle):
    n = 4096
    buf = torch.empty(n * CHUNK, dtype=torch.uint8, device="cuda")
    bt.fill_synthetic(buf.data_ptr(), n * CHUNK, 0, oracle.SEED_SYNTH)
    torch.cuda.synchronize()
    return buf


LAT = "lat"  # bt_sha1_set_latency_batch: the two-wave latency kernel (k_sha1_lat)
CHAIN = "chain"  # bt_sha1_set_chain_batch: one two-wave workgroup per chunk (k_sha1_chain)


@contextlib.contextmanager
def kernel_mode(bt, mode):
    """Pin the fixed-layout launches to one kernel: LAT, CHAIN, or the hot
    kernel (3 = its ring depth; latency and chain kernels off).  The product
    library has no other hot-kernel variant (the rejected ones are checked in
    tests/test_gpu_variants.py against the experiments build).  Restores the
    defaults."""
    prev = bt.set_latency_batch(1 << 62 if mode in (LAT, CHAIN) else 0)
    prev_chain = bt.set_chain_batch(1 << 62 if mode == CHAIN else 0)
    if mode not in (LAT, CHAIN):
        bt.set_variant(*(mode if isinstance(mode, tuple) else (mode, 1, 0)))
    try:
        yield
    finally:
        bt.set_variant(3, 1, 0)
        bt.set_latency_batch(prev)
        bt.set_chain_batch(prev_chain)


@pytest.mark.parametrize("variant", [(3, 1, 0), LAT, CHAIN])
def test_config2_4096_chunks_bit_exact(bt, torch, synth4096, variant):
    """BASELINE config 2: 4096 synthetic 512 KiB chunks, every digest == sha.c's,
    through each kernel of the product library a fixed-layout batch can run:
    the hot kernel, the latency kernel and the chain kernel."""
    with kernel_mode(bt, variant):
        n = 4096
        out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
        bt.chunks_dev(synth4096.data_ptr(), n, CHUNK, CHUNK, out.data_ptr())
        torch.cuda.synchronize()
        raw = out.cpu().numpy().tobytes()
        got = [(str(i), raw[20 * i:20 * i + 20].hex()) for i in range(n)]
        assert got == read_pairs("synth4096.txt")


@pytest.mark.parametrize("ring", [3, LAT, CHAIN])
def test_verify_dev_flags_mismatches(bt, torch, synth4096, ring):
    with kernel_mode(bt, ring):
        _verify_dev_flags_mismatches(bt, torch, synth4096)


def _verify_dev_flags_mismatches(bt, torch, synth4096):
    n = 1000
    golden = read_pairs("synth4096.txt")[:n]
    exp = bytearray(b"".join(bytes.fromhex(h) for _, h in golden))
    bad = {0, 17, 511, 999}
    for i in bad:
        exp[20 * i + (i % 20)] ^= 1
    d_exp = to_dev(torch, bytes(exp))
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    dig = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
    bt.verify_dev(synth4096.data_ptr(), n, CHUNK, CHUNK, d_exp.data_ptr(), ok.data_ptr(), dig.data_ptr())
    torch.cuda.synchronize()
    okl = ok.cpu().tolist()
    assert [i for i, v in enumerate(okl) if v == 0] == sorted(bad)
    assert all(v == 1 for i, v in enumerate(okl) if i not in bad)
    assert digests_of(torch, dig, 3)[2].hex() == golden[2][1]


@pytest.mark.parametrize("chunk_len,pitch,n", [
    (0, 16, 5), (1, 16, 3), (55, 64, 65), (56, 64, 64), (64, 64, 63), (100, 112, 129),
    (128, 128, 64), (192, 192, 65), (448, 448, 70), (4096 + 17, 4096 + 32, 130),
    (65536 + 63, 65536 + 64, 66), (3 * 128 * 5, 3 * 128 * 5, 200),
    (1000, 1003, 67),            # odd pitch -> generic kernel
    (CHUNK, CHUNK + 256, 65),    # padded pitch, fast kernel
])
@pytest.mark.parametrize("ring", [3, LAT, CHAIN])
def test_fixed_layouts_vs_oracle(bt, torch, oracle, chunk_len, pitch, n, ring):
    total = pitch * (n - 1) + chunk_len
    host = bytearray(oracle.fill_synthetic(total, 11, 0xC0FFEE))
    d = to_dev(torch, bytes(host))
    out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
    with kernel_mode(bt, ring):
        bt.chunks_dev(d.data_ptr(), n, chunk_len, pitch, out.data_ptr())
        torch.cuda.synchronize()
    want = [oracle.sha1(bytes(host[i * pitch:i * pitch + chunk_len])) for i in range(n)]
    assert digests_of(torch, out, n) == want


def _ragged_line_counts(bt, torch, oracle, ring):
    deepest = 4 if ring in (LAT, CHAIN) else ring
    for blocks in range(0, 2 * 2 * deepest + 3):
        for r in (0, 5, 56):
            L = 64 * blocks + r
            n = 70
            pitch = (L + 15) // 16 * 16 or 16
            host = bytearray(oracle.fill_synthetic(pitch * n, blocks, deepest))
            d = to_dev(torch, bytes(host))
            out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
            bt.chunks_dev(d.data_ptr(), n, L, pitch, out.data_ptr())
            torch.cuda.synchronize()
            got = digests_of(torch, out, n)
            for i in (0, 1, 63, 64, 69):
                assert got[i] == oracle.sha1(bytes(host[i * pitch:i * pitch + L])), (ring, L, i)


def test_every_kernel_on_ragged_line_counts(bt, torch, oracle):
    for ring in (3, LAT, CHAIN):
        with kernel_mode(bt, ring):
            _ragged_line_counts(bt, torch, oracle, ring)


def test_host_pipeline_c_tar_and_tail(bt, oracle):
    img = c_tar_bytes()
    got = [d.hex() for d in bt.chunks_host(img)]
    ref = [l.split()[1] for l in open(os.path.join(GOLDEN, "ref_C.chunks")).read().splitlines()[2:]]
    assert got == ref
    tail = bytes(oracle.fill_synthetic(3 * CHUNK + 12345, 0, oracle.SEED_TAIL))
    want = open(os.path.join(GOLDEN, "tail.make-chunks.out")).read()
    assert "".join(f"{i} {d.hex()}\n" for i, d in enumerate(bt.chunks_host(tail))) == want
    assert "".join(f"{i} {d.hex()}\n" for i, d in enumerate(bt.chunks_host(tail, ndev=0))) == want
    assert bt.chunks_host(b"") == []
    # many batches through the double-buffered pipeline (small chunks -> many per batch)
    big = bytes(oracle.fill_synthetic(5 * 1024 * 1024 + 77, 9, 9))
    assert bt.chunks_host(big, chunk_len=4096) == oracle.hash_chunks(big, 4096)


@pytest.mark.parametrize("variant", [(3, 1, 0), LAT, CHAIN])
def test_image_tail_in_same_launch(bt, oracle, variant):
    """launch_image: the short last chunk rides in the hot kernel's (or the
    latency kernel's) tail wave."""
    with kernel_mode(bt, variant):
        for chunk_len in (4096, 64 * 1024):
            for nfull in (0, 1, 63, 64, 65, 130):
                for rem in (1, 3, 55, 56, 63, 64, 65, 1000, chunk_len - 1):
                    img = bytes(oracle.fill_synthetic(nfull * chunk_len + rem, nfull + rem, 0x7A11))
                    assert bt.chunks_host(img, chunk_len=chunk_len) == oracle.hash_chunks(img, chunk_len), \
                        (variant, chunk_len, nfull, rem)


def test_make_chunks_file_api(bt, oracle, tmp_path):
    p = tmp_path / "C.tar"
    p.write_bytes(c_tar_bytes())
    assert "".join(f"{i} {d.hex()}\n" for i, d in enumerate(bt.make_chunks_file(str(p)))) == \
        open(os.path.join(GOLDEN, "C.tar.make-chunks.out")).read()
    e = tmp_path / "empty"
    e.write_bytes(b"")
    assert bt.make_chunks_file(str(e)) == []


def _libc():
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fdopen.restype = ctypes.c_void_p
    libc.fdopen.argtypes = [ctypes.c_int, ctypes.c_char_p]
    libc.fseek.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int]
    libc.feof.argtypes = [ctypes.c_void_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    return libc


def _chunks_fp(bt, fp, n):
    out = (ctypes.c_uint8 * (20 * max(n, 1)))()
    got = bt.lib.bt_sha1_chunks_file(ctypes.c_void_p(fp), CHUNK, out, n)
    assert got >= 0, bt.last_error()
    raw = bytes(out)
    return [raw[20 * i:20 * i + 20] for i in range(got)]


def test_file_path_threaded_reads_offsets_and_pipes(bt, oracle, tmp_path):
    """The FILE* path reads regular files with parallel preads from the FILE's
    logical position (several 16 MiB pieces per batch here) and leaves the
    stream at EOF like chunk.c's fread loop; pipes go through fread."""
    data = bytes(oracle.fill_synthetic(80 * 1024 * 1024 + 12345, 21, 0xF11E))
    p = tmp_path / "big.bin"
    p.write_bytes(data)
    libc = _libc()
    want = oracle.hash_chunks(data, CHUNK)
    fp = libc.fopen(str(p).encode(), b"rb")
    try:
        assert _chunks_fp(bt, fp, len(want)) == want
        assert libc.feof(fp) != 0
    finally:
        libc.fclose(fp)
    off = 3 * CHUNK + 100  # a caller that already consumed part of the stream
    fp = libc.fopen(str(p).encode(), b"rb")
    try:
        assert libc.fseek(fp, off, 0) == 0
        assert _chunks_fp(bt, fp, len(want)) == oracle.hash_chunks(data[off:], CHUNK)
        assert libc.feof(fp) != 0
    finally:
        libc.fclose(fp)
    rfd, wfd = os.pipe()

    def writer():
        with os.fdopen(wfd, "wb") as w:
            w.write(data)

    t = threading.Thread(target=writer)
    t.start()
    fp = libc.fdopen(rfd, b"rb")
    try:
        assert _chunks_fp(bt, fp, len(want)) == want
    finally:
        libc.fclose(fp)
        t.join()


def test_chunks_host_pageable_parallel_staging(bt, oracle):
    """Pageable input > 32 MiB: the staging copy into pinned memory is split
    over threads; digests unchanged."""
    data = bytes(oracle.fill_synthetic(96 * 1024 * 1024 + 999, 22, 0xF11F))
    assert bt.chunks_host(data) == oracle.hash_chunks(data, CHUNK)


def test_make_chunks_cli(tmp_path, oracle):
    exe = os.path.join(PKG, "bin", "make-chunks")
    p = tmp_path / "C.tar"
    p.write_bytes(c_tar_bytes())
    out = subprocess.run([exe, str(p)], capture_output=True, check=True).stdout.decode()
    assert out == open(os.path.join(GOLDEN, "C.tar.make-chunks.out")).read()
    out_g = subprocess.run([exe, "-g", "0", "-m", str(p)], capture_output=True, check=True).stdout.decode()
    assert out_g == f"File: {p}\nChunks:\n" + out
    t = tmp_path / "tail.bin"
    t.write_bytes(bytes(oracle.fill_synthetic(3 * CHUNK + 12345, 0, oracle.SEED_TAIL)))
    out_t = subprocess.run([exe, str(t)], capture_output=True, check=True).stdout.decode()
    assert out_t == open(os.path.join(GOLDEN, "tail.make-chunks.out")).read()


def test_reference_make_chunks_linked_to_dropin(tmp_path):
    """The reference's own make_chunks.c, unchanged, linked against libbtsha1.so
    (built in the build container into oracle/_ref/make-chunks-dropin)."""
    exe = os.path.join(REPO, "oracle", "_ref", "make-chunks-dropin")
    if not os.path.exists(exe):
        pytest.skip("drop-in reference binary not built")
    p = tmp_path / "C.tar"
    p.write_bytes(c_tar_bytes())
    env = dict(os.environ, LD_LIBRARY_PATH=PKG + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    out = subprocess.run([exe, str(p)], capture_output=True, check=True, env=env).stdout.decode()
    assert out == open(os.path.join(GOLDEN, "C.tar.make-chunks.out")).read()


@pytest.mark.parametrize("size", [0, 1, 55, 56, 63, 64, 65, CHUNK - 1, CHUNK, CHUNK + 1, 3 * CHUNK + 12345,
                                  33 * CHUNK - 7, 64 * CHUNK + 64 * 1024 + 56, 200 * CHUNK + 1])
def test_make_chunks_three_ways_on_random_sizes(tmp_path, oracle, size):
    """make-chunks stdout, byte for byte, three ways on the same file: the
    reference binary itself (make_chunks.c + chunk.c + sha.c on the CPU,
    oracle/_ref/make-chunks), the reference's make_chunks.c linked to
    libbtsha1.so (oracle/_ref/make-chunks-dropin) and our CLI -- sizes around
    the MD padding boundaries (55/56/63/64 bytes into a block) and the chunk
    boundary, with short last chunks riding in the same launch (chunk.c:20)."""
    ref = os.path.join(REPO, "oracle", "_ref", "make-chunks")
    dropin = os.path.join(REPO, "oracle", "_ref", "make-chunks-dropin")
    ours = os.path.join(PKG, "bin", "make-chunks")
    for exe in (ref, dropin):
        assert os.path.exists(exe), f"{exe} missing: built by oracle/Makefile / make dropin where the reference exists"
    p = tmp_path / "f.bin"
    p.write_bytes(bytes(oracle.fill_synthetic(size, size, 0x3A4E)))
    env = dict(os.environ, LD_LIBRARY_PATH=PKG + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    outs = [subprocess.run([exe, str(p)], capture_output=True, check=True, env=env).stdout for exe in (ref, dropin, ours)]
    assert outs[0] == outs[1] == outs[2], size
    assert outs[0].count(b"\n") == (size + CHUNK - 1) // CHUNK


def test_reference_save_chunk_linked_to_dropin(tmp_path):
    """Caller #2 at the boundary: the reference peer's own util.c (save_data_packet
    util.c:250-277 + save_chunk util.c:304-337) and file.c, compiled unmodified
    and linked against libbtsha1.so in place of chunk.o + sha.o (reference
    Makefile:6), receive C.tar's four chunks as 1484-byte DATA payloads; chunk
    2 arrives corrupted first.  Exactly one "Verification failed!", the failed
    chunk goes back to NOT_STARTED (common.h: 2), every chunk ends OWNED (0)
    and the written file is C.tar byte for byte (util.c:322-323)."""
    exe = os.path.join(REPO, "oracle", "_ref", "save-chunk-dropin")
    assert os.path.exists(exe), "built by `make dropin` in the build container (needs the reference sources)"
    data = tmp_path / "C.tar"
    data.write_bytes(c_tar_bytes())
    has = tmp_path / "has.chunks"
    has.write_text("")
    out = tmp_path / "out.tar"
    env = dict(os.environ, LD_LIBRARY_PATH=PKG + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([exe, "-c", "2", str(data), os.path.join(GOLDEN, "ref_C.chunks"),
                        os.path.join(GOLDEN, "C.tar.make-chunks.out"), str(has), str(out)],
                       capture_output=True, env=env, timeout=120)
    text = r.stdout.decode()
    assert r.returncode == 0, (text[-2000:], r.stderr.decode()[-2000:])
    assert text.count("Verification failed!") == 1
    states = [tuple(map(int, l.split()[1:])) for l in text.splitlines() if l.startswith("STATE ")]
    assert states == [(0, 0), (1, 0), (2, 2), (2, 0), (3, 0)], states
    assert "ALL_FINISHED 1" in text
    assert out.read_bytes() == data.read_bytes()


def test_verify_stream_cli(tmp_path):
    exe = os.path.join(PKG, "bin", "verify-stream")
    p = tmp_path / "C.tar"
    p.write_bytes(c_tar_bytes())
    ck = os.path.join(GOLDEN, "ref_C.chunks")
    r = subprocess.run([exe, "-b", "3", str(p), ck], capture_output=True, text=True, check=True)
    assert '"ok": 4, "failed": 0' in r.stdout and "Verification failed" not in r.stdout
    r = subprocess.run([exe, "-b", "2", "-x", str(p), ck], capture_output=True, text=True, check=True)
    assert r.stdout.count("Verification failed!") == 1 and '"failed": 1' in r.stdout


def test_verifier_async_batches(bt, oracle):
    img = c_tar_bytes()
    chunks = [img[i * CHUNK:(i + 1) * CHUNK] for i in range(4)]
    ref = [bytes.fromhex(l.split()[1]) for l in open(os.path.join(GOLDEN, "ref_C.chunks")).read().splitlines()[2:]]
    v = bt.Verifier(batch=5, nstreams=2)
    results, want = [], []
    for k in range(23):
        exp = ref[k % 4] if k % 6 else bytes(20)  # every 6th expectation is wrong
        if k % 2:
            v.submit(chunks[k % 4], exp, tag=1000 + k)
        else:
            v.slot_fill(chunks[k % 4], exp, tag=1000 + k)
        want.append((1000 + k, k % 6 != 0, ref[k % 4]))
        results += v.poll()
    results += v.drain()
    assert v.pending() == 0
    assert results == want
    with pytest.raises(bt.BtSha1Error):
        v.submit(b"short", ref[0], tag=1)
    v.close()


def test_verifier_column_split_batches(bt, oracle):
    """Verifier batches of >= 256 MiB are copied and hashed column by column
    (the verdicts come ~0.9 ms after the last byte instead of one chunk's
    hash): 1100 distinct chunks in batches of 512 -- two split batches, a
    76-chunk one that is not -- with every 97th expectation wrong and a few
    slots released unverified; verdicts and digests exact, in order."""
    import numpy as np
    n = 1100
    img = np.empty(n * CHUNK, dtype=np.uint8)
    img.view(np.uint64)[:] = np.arange(img.size // 8, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C35)
    ref = oracle.hash_chunks(img, CHUNK, nthreads=8)
    v = bt.Verifier(batch=512, nstreams=2)
    want, got = [], []
    for k in range(n):
        chunk = img[k * CHUNK:(k + 1) * CHUNK]
        if k % 211 == 5:  # an aborted download: the slot goes back unverified
            v.release(v.slot())
        exp = ref[k] if k % 97 else bytes(20)
        v.slot_fill(chunk, exp, tag=k)
        want.append((k, k % 97 != 0, ref[k]))
        got += v.poll()
    got += v.drain()
    v.close()
    assert len(got) == n and got == want


def test_verifier_lifecycle_and_staging_growth(bt, oracle):
    """Verifiers created and destroyed repeatedly (their chunk slots are
    page-locked staging memory, registered and unregistered each time) and
    host pipelines whose staging grows between calls keep exact results."""
    img = c_tar_bytes()
    chunks = [img[i * CHUNK:(i + 1) * CHUNK] for i in range(4)]
    ref = [oracle.sha1(c) for c in chunks]
    for batch, streams in ((1, 2), (7, 3), (4, 2), (16, 4), (2, 2)):
        v = bt.Verifier(batch=batch, nstreams=streams)
        for k in range(9):
            v.slot_fill(chunks[k % 4], ref[k % 4] if k != 5 else bytes(20), tag=k)
        got = v.drain()
        v.close()
        assert got == [(k, k != 5, ref[k % 4]) for k in range(9)], (batch, streams)
    for mib in (1, 3, 70, 9):  # staging sized by the input, grow-only
        data = (img * (mib // 2 + 1))[:mib * 1024 * 1024 + 777]
        want = [oracle.sha1(data[o:o + CHUNK]) for o in range(0, len(data), CHUNK)]
        assert bt.chunks_host(data) == want, mib


def test_config4_every_digest_equals_the_reference(bt, torch):
    """BASELINE config 4's whole workload -- 1,048,576 x 512 KiB chunks, 512
    GiB, the 8-GPU split's eight rank slices [r*131072, (r+1)*131072) --
    hashed slice after slice on this one GPU (512 GiB does not fit in one
    GPU's HBM at once): the checksum of all 1,048,576 digests in global order
    equals the REFERENCE's (tests/golden/synth_checksums.txt, sha.c's digests
    of the same chunks), and so does every rank-count prefix the N = 1, 2 and
    4 lines compare with.  What the driver's N = 8 line reports as
    parity_all_vs_golden, checked here on hardware ahead of it."""
    table = dict(read_pairs("synth_checksums.txt"))
    per, ranks = 131072, 8
    buf = torch.empty(per * CHUNK, dtype=torch.uint8, device="cuda")
    dig = torch.empty(20 * per, dtype=torch.uint8, device="cuda")
    h = hashlib.sha1()
    for r in range(ranks):
        bt.fill_synthetic(buf.data_ptr(), per * CHUNK, r * per * (CHUNK // 8), 0x0B175EED)
        bt.chunks_dev(buf.data_ptr(), per, CHUNK, CHUNK, dig.data_ptr())
        torch.cuda.synchronize()
        h.update(dig.cpu().numpy().tobytes())
        if str((r + 1) * per) in table:
            assert h.copy().hexdigest() == table[str((r + 1) * per)], (r + 1) * per
    assert h.hexdigest() == table["1048576"]


def test_full_size_config3_properties(bt, torch, oracle):
    """BASELINE config 3 size (131072 x 512 KiB = 64 GiB in HBM): EVERY digest
    equal to the oracle's on the chunk regenerated on the host (threaded C
    sweep, oracle.synth_digests), plus determinism, distinctness and the
    reference's golden digests for the first 4096."""
    n = 131072
    try:
        buf = torch.empty(n * CHUNK, dtype=torch.uint8, device="cuda")
    except RuntimeError:
        pytest.skip("not enough device memory")
    bt.fill_synthetic(buf.data_ptr(), n * CHUNK, 0, oracle.SEED_SYNTH)
    out = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
    bt.chunks_dev(buf.data_ptr(), n, CHUNK, CHUNK, out.data_ptr())
    out2 = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
    bt.chunks_dev(buf.data_ptr(), n, CHUNK, CHUNK, out2.data_ptr())
    torch.cuda.synchronize()
    del buf
    raw = out.cpu().numpy().tobytes()
    assert raw == out2.cpu().numpy().tobytes()
    dig = [raw[20 * i:20 * i + 20] for i in range(n)]
    assert len(set(dig)) == n
    golden = read_pairs("synth4096.txt")
    assert [d.hex() for d in dig[:4096]] == [h for _, h in golden]
    sample = list(range(n - 64, n)) + list(range(4096, n, 1024))
    for i in sample:
        assert dig[i] == oracle.sha1(bytes(oracle.fill_synthetic(CHUNK, i * 65536, oracle.SEED_SYNTH))), i
    want = oracle.synth_digests(0, n)  # all 131072, ~10 s on the box's 16 CPUs
    bad = [i for i in range(n) if raw[20 * i:20 * i + 20] != want[20 * i:20 * i + 20]]
    assert not bad, (len(bad), bad[:10])


def test_pipeline_stats_account_for_each_host_run(bt, oracle, tmp_path):
    """bt_sha1_get_pipeline_stats after each kind of host pipeline run on
    this thread: chunk and byte counts, batches, how the input was fed
    (pageable >= 64 MiB: page-locked batch by batch; pinned: direct DMA; a
    file: staged reads), a phase split that fits inside the call, and the
    NUMA placement (under the default policy on a multi-node box the staging
    lanes sit on the GPU's node)."""
    import numpy as np
    data = np.frombuffer(bytes(oracle.fill_synthetic(150 * CHUNK + 999, 7, 0x57A7)), dtype=np.uint8).copy()
    want = b"".join(oracle.hash_chunks(bytes(data), CHUNK))
    addr = data.ctypes.data
    t0 = time.perf_counter()
    assert bt.chunks_host_addr(addr, data.nbytes) == want
    wall = time.perf_counter() - t0
    s = bt.pipeline_stats()
    assert (s["chunks"], s["bytes"], s["feed"], s["staged"]) == (151, data.nbytes, "registered", False)
    # two batches of 76 chunks (the input's halves); 76 chunks are too few for
    # the column-split tail (under 256 MiB)
    assert s["column_chunks"] == 0 and s["batches"] == 2 and s["batch_bytes"] == 76 * CHUNK
    assert s["registered_batches"] == 2 and s["register_s"] >= 0
    assert 0 < s["total_s"] <= wall and s["fill_s"] + s["wait_s"] + s["alloc_s"] <= s["total_s"] * 1.001
    assert sum(s["src_pages"]) > 0 and sum(s["copy_pieces"]) == 0   # nothing copied by the staging threads
    bt.host_register(addr, data.nbytes)  # nothing of the call left registered
    try:
        assert bt.chunks_host_addr(addr, data.nbytes) == want
        d = bt.pipeline_stats()
        assert (d["chunks"], d["feed"], d["numa_policy"], d["registered_batches"]) == (151, "direct", "none", 0)
        assert d["column_chunks"] == 0 and d["batches"] == 2
        assert sum(d["copy_pieces"]) == 0 and sum(d["lane_pages"]) == 0
    finally:
        bt.host_unregister(addr)
    f = tmp_path / "img"
    f.write_bytes(data.tobytes())
    assert b"".join(bt.make_chunks_file(str(f))) == want
    m = bt.pipeline_stats()
    assert (m["chunks"], m["bytes"], m["feed"]) == (151, data.nbytes, "staged")
    assert sum(m["lane_pages"]) > 0 and sum(m["copy_pieces"]) > 0
    if m["numa_policy"] in ("lanes", "gpu"):
        assert m["lane_pages"][m["gpu_numa_node"]] == sum(m["lane_pages"])
    if m["numa_policy"] == "gpu":
        assert m["copy_pieces"][m["gpu_numa_node"]] == sum(m["copy_pieces"])


def test_pageable_image_registered_batch_by_batch_at_every_alignment(bt, oracle):
    """The registered feed locks the whole pages of each batch and sends the
    unaligned head / tail bytes through a small pinned edge buffer: images
    starting on a page, 1, 16 and 4095 bytes past one, with a short last
    chunk, hash exactly; no page stays registered after the call (the caller
    can register the image itself afterwards)."""
    import numpy as np
    n = 140 * CHUNK + 12345
    raw = np.frombuffer(bytes(oracle.fill_synthetic(n + 3 * 4096, 9, 0xA11C)), dtype=np.uint8).copy()
    base = raw.ctypes.data
    first_page = (-base) % 4096
    for shift in (first_page, first_page + 1, first_page + 16, first_page + 4095):
        addr = base + shift
        want = b"".join(oracle.hash_chunks(bytes(raw[shift:shift + n]), CHUNK))
        assert bt.chunks_host_addr(addr, n) == want, shift
        s = bt.pipeline_stats()
        # two batches of 71 chunks, each locking its whole pages
        assert (s["feed"], s["registered_batches"], s["chunks"], s["column_chunks"]) == ("registered", 2, 141, 0), \
            shift
        bt.host_register(addr, n)
        bt.host_unregister(addr)


def test_registered_feed_falls_back_to_staging_pages_it_cannot_lock(bt, oracle, tmp_path):
    """Pages the registered feed cannot lock -- part of the image registered
    by the caller already, or a read-only file mapping -- are staged through
    the lane instead: exact digests either way, and the caller's own
    registration is left as it was."""
    import numpy as np
    n = 150 * CHUNK
    data = np.frombuffer(bytes(oracle.fill_synthetic(n, 21, 0xFA11)), dtype=np.uint8).copy()
    want = b"".join(oracle.hash_chunks(bytes(data), CHUNK))
    addr = data.ctypes.data
    mid = addr + ((40 * CHUNK + 4095) & ~4095)
    bt.host_register(mid, 8 * CHUNK)   # the caller's own registration inside batch 0
    try:
        assert bt.chunks_host_addr(addr, n) == want
        assert bt.pipeline_stats()["feed"] == "registered"
    finally:
        bt.host_unregister(mid)        # still the caller's, still there
    f = tmp_path / "ro.img"
    f.write_bytes(data.tobytes())
    ro = np.memmap(str(f), dtype=np.uint8, mode="r")
    assert bt.chunks_host_addr(ro.ctypes.data, n) == want
    del ro


# 130 chunks + 77 bytes from 5 bytes past a page: the split tail is the last
# 66 chunks; with the registered feed chunks 65..128 go by columns (chunk 129
# reaches the input's last, partial page and, like the short one, is hashed
# from a pinned copy), with the caller's own registration (direct feed) 65..129.
@pytest.mark.parametrize("env,feed,cols,cols_direct", [
    ({"BT_SHA1_PAGEABLE": "stage"}, "staged", 65, 65),  # staged: no page constraint, only the short chunk left over
    ({"BT_SHA1_COLUMNS": "0"}, "registered", 0, 0),
    ({}, "registered", 64, 65),
    ({"BT_SHA1_COLUMNS": "2"}, "registered", 64, 65),
    ({"BT_SHA1_COLUMNS": "16"}, "registered", 64, 65),
    ({"BT_SHA1_COLUMNS": "3"}, "registered", 0, 0),  # no 3-way split of 512 KiB into whole blocks: off
    ({"BT_SHA1_COLUMN_MIN_MB": "256"}, "registered", 0, 0)])
def test_pageable_feed_knobs(tmp_path, env, feed, cols, cols_direct):
    """BT_SHA1_PAGEABLE=stage: pageable input of any size is copied into the
    staging lanes, as before round 6 (its split tail's columns gathered there
    by the copy threads); BT_SHA1_COLUMNS sets the columns of the
    column-split tail (0 = off; a count that does not split the chunk into
    whole 64-byte blocks turns it off) and BT_SHA1_COLUMN_MIN_MB the smallest
    part it takes (0 here unless given).  Child processes: the knobs are read
    once.  Exact digests, pageable and then registered by the caller."""
    code = (
        "import sys, numpy as np; sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2]);"
        "import btsha1 as bt, py_oracle as o;"
        "raw = np.frombuffer(bytes(o.fill_synthetic(130 * 524288 + 77 + 4096, 3, 0x5EED)), dtype=np.uint8).copy();"
        "k = (-raw.ctypes.data) % 4096 + 5; d = raw[k:k + 130 * 524288 + 77];"
        "w = b''.join(o.hash_chunks(bytes(d), 524288));"
        "assert bt.chunks_host_addr(d.ctypes.data, d.nbytes) == w;"
        "s = bt.pipeline_stats();"
        "bt.host_register(d.ctypes.data, d.nbytes);"
        "assert bt.chunks_host_addr(d.ctypes.data, d.nbytes) == w;"
        "t = bt.pipeline_stats(); bt.host_unregister(d.ctypes.data);"
        "print('feed', s['feed'], 'cols', s['column_chunks'], 'chunks', s['chunks'], 'pieces', sum(s['copy_pieces']),"
        "      'dfeed', t['feed'], 'dcols', t['column_chunks'], 'dchunks', t['chunks'])")
    r = subprocess.run([sys.executable, "-c", code, PKG, os.path.join(REPO, "oracle")], capture_output=True,
                       text=True, env=dict(os.environ, **{"BT_SHA1_COLUMN_MIN_MB": "0", **env}), timeout=120)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-2000:])
    out = r.stdout.split()
    got = dict(zip(out[::2], out[1::2]))
    assert (got["feed"], int(got["cols"]), int(got["chunks"])) == (feed, cols, 131), r.stdout
    assert (got["dfeed"], int(got["dcols"]), int(got["dchunks"])) == ("direct", cols_direct, 131), r.stdout
    assert (int(got["pieces"]) > 0) == (feed == "staged")


def test_column_split_tail_at_full_size(bt, oracle):
    """The column-split tail at its default threshold: 1100 chunks + 333 bytes
    (550 MiB) pageable from an unaligned start, the same bytes registered by
    the caller (direct DMA), and staged; at chunk sizes of 512, 256, 192 and
    64 KiB: the last ~half goes by columns (275 MiB), digests exact against
    the oracle, stats say so."""
    import numpy as np
    n = 1100 * CHUNK + 333
    raw = np.empty(n + 4096 - n % 8, dtype=np.uint8)
    raw.view(np.uint64)[:] = np.arange(raw.size // 8, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    d = raw[100:100 + n]
    # 512 / 256 KiB, the smallest chunk the split takes (64 KiB: 4 KiB columns,
    # 4400 rows), and one that is no power of two (192 KiB: 24 KiB columns)
    for cl in (CHUNK, CHUNK // 2, 65536, 196608):
        want = b"".join(oracle.hash_chunks(d, cl, nthreads=8))
        nch = (n + cl - 1) // cl
        assert bt.chunks_host_addr(d.ctypes.data, n, chunk_len=cl) == want, cl
        s = bt.pipeline_stats()
        assert (s["feed"], s["chunks"]) == ("registered", nch) and (nch // 2 - 2) <= s["column_chunks"] <= nch // 2, s
        bt.host_register(d.ctypes.data, n)
        try:
            assert bt.chunks_host_addr(d.ctypes.data, n, chunk_len=cl) == want, cl
            t = bt.pipeline_stats()
            assert (t["feed"], t["chunks"], t["column_chunks"]) == ("direct", nch, (nch + 1) // 2 - 1), t
        finally:
            bt.host_unregister(d.ctypes.data)
        prev = bt.set_pageable_feed("stage")  # the copy threads gather the columns into the staging lane
        try:
            assert bt.chunks_host_addr(d.ctypes.data, n, chunk_len=cl) == want, cl
            u = bt.pipeline_stats()
            assert (u["feed"], u["chunks"], u["column_chunks"]) == ("staged", nch, (nch + 1) // 2 - 1), u
            assert u["fill_s"] > 0 and sum(u["copy_pieces"]) > 0
        finally:
            bt.set_pageable_feed(prev)


def test_registered_host_image_direct_dma(bt, oracle):
    import numpy as np
    data = np.frombuffer(bytes(oracle.fill_synthetic(9 * CHUNK + 777, 5, 0xD1A), ), dtype=np.uint8).copy()
    want = b"".join(oracle.hash_chunks(bytes(data), CHUNK))
    addr = data.ctypes.data
    assert bt.chunks_host_addr(addr, data.nbytes) == want          # pageable: staged
    bt.host_register(addr, data.nbytes)
    try:
        assert bt.chunks_host_addr(addr, data.nbytes) == want      # pinned: direct DMA
        assert bt.chunks_host_addr(addr, data.nbytes, ndev=0) == want
    finally:
        bt.host_unregister(addr)


def test_verify_stream_zero_copy_mode(tmp_path):
    exe = os.path.join(PKG, "bin", "verify-stream")
    p = tmp_path / "C.tar"
    p.write_bytes(c_tar_bytes())
    ck = os.path.join(GOLDEN, "ref_C.chunks")
    r = subprocess.run([exe, "-z", "-b", "8", "-s", "3", "-r", "3", str(p), ck], capture_output=True, text=True, check=True)
    assert '"chunks": 72, "ok": 72, "failed": 0' in r.stdout


@pytest.mark.parametrize("batch,streams,nchunks", [(64, 2, 128), (32, 3, 48), (16, 2, 32)])
def test_verify_stream_zero_copy_distinct_chunks(tmp_path, oracle, batch, streams, nchunks):
    """-z with as many DISTINCT chunks as the ring has slots (bench.py's
    host_path leg runs 2048 at batch 1024 x 2): after round 0's drain the
    verifier resumes at whichever batch is next, so each later commit must be
    paired with the chunk resident in the slot it gets, not with slot order."""
    exe = os.path.join(PKG, "bin", "verify-stream")
    img = bytes(oracle.fill_synthetic(nchunks * CHUNK, 3, 0xFEED))
    p = tmp_path / "img"
    p.write_bytes(img)
    ck = tmp_path / "img.chunks"
    ck.write_text("".join(f"{i} {d.hex()}\n" for i, d in enumerate(oracle.hash_chunks(img, CHUNK))))
    r = subprocess.run([exe, "-z", "-b", str(batch), "-s", str(streams), "-r", "4", str(p), str(ck)],
                       capture_output=True, text=True, timeout=120)
    ring = batch * max(streams, 2)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-500:])
    assert f'"chunks": {4 * ring}, "ok": {4 * ring}, "failed": 0' in r.stdout


@pytest.mark.parametrize("g", [2, 3])
def test_verify_stream_chunks_dealt_modulo_g_verifiers(tmp_path, oracle, g):
    """SURVEY.md §8e's streaming-verify split: -g G verifiers (one per GPU on
    a node; here G sharing this box's one GPU), received chunk id -> verifier
    id % G, chunks arriving interleaved across them.  Packetized receive with
    every 7th chunk corrupted (-x): exactly those fail, whatever G; zero-copy
    receive (-z): every commit of every verifier's ring verifies."""
    exe = os.path.join(PKG, "bin", "verify-stream")
    n = 12 * g
    img = bytes(oracle.fill_synthetic(n * CHUNK, 11, 0xFEED))
    p = tmp_path / "img"
    p.write_bytes(img)
    ck = tmp_path / "img.chunks"
    ck.write_text("".join(f"{i} {d.hex()}\n" for i, d in enumerate(oracle.hash_chunks(img, CHUNK))))
    r = subprocess.run([exe, "-g", str(g), "-b", "4", "-s", "2", "-x", str(p), str(ck)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-500:])
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    bad = sum(1 for k in range(n) if k % 7 == 3)
    assert (summary["chunks"], summary["ok"], summary["failed"], summary["verifiers"]) == (n, n - bad, bad, g)
    assert r.stdout.count("Verification failed!") == bad
    # zero-copy: each verifier's chunk count (12) divides its ring (4 x 3)
    r = subprocess.run([exe, "-g", str(g), "-z", "-b", "4", "-s", "3", "-r", "3", str(p), str(ck)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-500:])
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert (summary["chunks"], summary["ok"], summary["failed"]) == (3 * 12 * g, 3 * 12 * g, 0)


@pytest.mark.parametrize("g", [2, 4])
def test_verify_stream_receive_threads_and_warmup_rounds(tmp_path, oracle, g):
    """-t: every verifier gets a receive thread of its own (the packetized
    util.c:275 copies of the G verifiers run side by side); -w: untimed
    warm-up rounds.  Every 7th chunk corrupted (-x) fails in every round,
    exactly those; the summary counts the timed rounds only."""
    exe = os.path.join(PKG, "bin", "verify-stream")
    n = 8 * g
    img = bytes(oracle.fill_synthetic(n * CHUNK, 17, 0xFEED))
    p = tmp_path / "img"
    p.write_bytes(img)
    ck = tmp_path / "img.chunks"
    ck.write_text("".join(f"{i} {d.hex()}\n" for i, d in enumerate(oracle.hash_chunks(img, CHUNK))))
    r = subprocess.run([exe, "-g", str(g), "-t", "-b", "3", "-s", "2", "-r", "3", "-w", "1", "-x", str(p), str(ck)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-500:])
    s = json.loads(r.stdout.strip().splitlines()[-1])
    bad = 3 * sum(1 for k in range(n) if k % 7 == 3)
    assert (s["chunks"], s["ok"], s["failed"], s["verifiers"], s["receive_threads"]) == (3 * n, 3 * n - bad, bad, g, g)
    assert (s["timed_chunks"], s["warmup_rounds"], s["late_fills"]) == (2 * n, 1, 0)
    assert r.stdout.count("Verification failed!") == bad
    # zero-copy with receive threads: every commit of every ring verifies
    r = subprocess.run([exe, "-g", str(g), "-t", "-z", "-b", "4", "-s", "2", "-r", "4", str(p), str(ck)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-500:])
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert (s["chunks"], s["ok"], s["failed"], s["timed_chunks"]) == (4 * 8 * g, 4 * 8 * g, 0, 3 * 8 * g)
    # no timed round left: refused before any GPU work
    r = subprocess.run([exe, "-r", "2", "-w", "2", str(p), str(ck)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 255 and "no timed round" in r.stderr


def test_verifier_concurrent_downloads_out_of_order(bt):
    """A peer assembles up to max_conn chunks at once (util.c:250-277); slots
    are committed in completion order, some downloads abort (released)."""
    import ctypes
    rng = random.Random(5)
    img = c_tar_bytes()
    chunks = [img[i * CHUNK:(i + 1) * CHUNK] for i in range(4)]
    ref = [bytes.fromhex(l.split()[1]) for l in open(os.path.join(GOLDEN, "ref_C.chunks")).read().splitlines()[2:]]
    v = bt.Verifier(batch=4, nstreams=6)
    active, want, got = [], {}, []
    for k in range(40):
        p = v.slot()
        ctypes.memmove(p, chunks[k % 4], CHUNK)
        active.append((p, k))
        while len(active) >= 4 or (k == 39 and active):      # complete a random in-flight download
            p2, k2 = active.pop(rng.randrange(min(2, len(active))))  # one of the two oldest
            if k2 % 9 == 4:
                v.release(p2)                                # aborted download: no verdict
            else:
                exp = ref[k2 % 4] if k2 % 5 else ref[(k2 + 1) % 4]
                v.commit(p2, exp, tag=k2)
                want[k2] = (k2 % 5 != 0)
            got += v.poll()
    got += v.drain()
    assert {t: ok for t, ok, _ in got} == want
    assert all(d == ref[t % 4] for t, _, d in got)
    with pytest.raises(bt.BtSha1Error):
        v.commit(12345, ref[0], tag=0)                     # not an outstanding slot
    v.close()


def test_host_runtime_under_asan(tmp_path):
    """Host-side ASan/UBSan build of the C runtime (verifier ring, pipelines,
    streaming API) driven by tests/native/host_stress.c on the GPU."""
    exe = os.path.join(REPO, "build_variants", "asan", "host_stress")
    # built beforehand (`make all` / __graft_entry__.build()), never on the GPU box
    assert os.path.exists(exe), "build_variants/asan/host_stress missing: run `make asan` first"
    p = tmp_path / "C.tar"
    p.write_bytes(c_tar_bytes())
    ref = [l.split()[1] for l in open(os.path.join(GOLDEN, "ref_C.chunks")).read().splitlines()[2:]]
    # every registered-feed case with a 512-byte-multiple chunk size takes the
    # column-split tail (BT_SHA1_COLUMN_MIN_MB=0: however small the part)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", BT_SHA1_COLUMN_MIN_MB="0")
    r = subprocess.run([exe, str(p)] + ref,
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "ok (0 failures)" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def _dev_bytes(torch, b):
    t = torch.zeros(max(len(b), 4), dtype=torch.uint8, device="cuda")
    if b:
        t[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
    return t


@pytest.mark.parametrize("n_table,n_query", [(0, 5), (1, 3), (4, 4), (1000, 3000), (300000, 200000)])
def test_digest_lookup_matches_first_match_scan(bt, torch, n_table, n_query):
    """get_chunk_id (util.c:28-39): index of the FIRST equal digest, else -1."""
    import hashlib
    rng = random.Random(n_table)
    distinct = [hashlib.sha1(str(i).encode()).digest() for i in range(max(1, n_table // 2 + 1))]
    table = [distinct[rng.randrange(len(distinct))] for _ in range(n_table)]  # with duplicates
    absent = [hashlib.sha1(b"absent" + str(i).encode()).digest() for i in range(50)]
    queries = [(table[rng.randrange(n_table)] if n_table and rng.random() < 0.8 else absent[rng.randrange(50)])
               for _ in range(n_query)]
    first = {}
    for i, d in enumerate(table):
        first.setdefault(d, i)
    dt, dq = _dev_bytes(torch, b"".join(table)), _dev_bytes(torch, b"".join(queries))
    out = torch.full((n_query,), 7, dtype=torch.int64, device="cuda")
    bt.lookup_dev(dt.data_ptr(), n_table, dq.data_ptr(), n_query, out.data_ptr())
    torch.cuda.synchronize()
    assert out.cpu().tolist() == [first.get(q, -1) for q in queries]


@pytest.mark.parametrize("n_table", [1, 1000, 20000])
def test_digest_lookup_matches_the_reference_get_chunk_id(bt, torch, tmp_path, n_table):
    """Differential against the reference itself: util.c's get_chunk_id
    (util.c:28-39, compiled unmodified into oracle/_ref/chunks-ref) over a
    master file it parsed (util.c:113-164) with duplicate digests and
    shuffled ids, against bt_sha1_lookup_dev on the same table -- the id of
    the FIRST matching entry, or -1 for a miss."""
    import hashlib
    exe = os.path.join(REPO, "oracle", "_ref", "chunks-ref")
    assert os.path.exists(exe), "oracle/_ref/chunks-ref missing: build it with `make -C oracle` where the reference exists"
    rng = random.Random(1000 + n_table)
    distinct = [hashlib.sha1(b"t" + str(i).encode()).digest() for i in range(max(1, n_table * 2 // 3))]
    table = [distinct[rng.randrange(len(distinct))] for _ in range(n_table)]
    ids = list(range(n_table))
    rng.shuffle(ids)
    master = tmp_path / "m.chunks"
    master.write_text("File: x.tar\nChunks:\n" + "".join(f"{i} {h.hex()}\n" for i, h in zip(ids, table)))
    queries = [table[rng.randrange(n_table)] if rng.random() < 0.7 else hashlib.sha1(b"q" + str(k).encode()).digest()
               for k in range(3000)]
    qf = tmp_path / "q.txt"
    qf.write_text("".join(q.hex() + "\n" for q in queries))
    ref = [int(x) for x in subprocess.run([exe, "lookup", str(master), str(qf)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    name, entries = bt.parse_master(str(master))
    dt = _dev_bytes(torch, b"".join(h for _, h in entries))
    dq = _dev_bytes(torch, b"".join(queries))
    out = torch.full((len(queries),), 7, dtype=torch.int64, device="cuda")
    bt.lookup_dev(dt.data_ptr(), len(entries), dq.data_ptr(), len(queries), out.data_ptr())
    torch.cuda.synchronize()
    got = [entries[i][0] if i >= 0 else -1 for i in out.cpu().tolist()]
    assert len(ref) == len(queries) and got == ref


def test_parse_then_lookup_then_verify_c_tar(bt, torch):
    """The peer's flow on the reference fixtures: master file -> GPU lookup of
    the has-file hashes -> verify the C.tar chunks against the master."""
    name, master = bt.parse_master(os.path.join(GOLDEN, "ref_C.chunks"))
    has = bt.parse_chunk_list(os.path.join(GOLDEN, "ref_B.chunks"))
    dt = _dev_bytes(torch, b"".join(h for _, h in master))
    dq = _dev_bytes(torch, b"".join(h for _, h in has))
    out = torch.zeros(len(has), dtype=torch.int64, device="cuda")
    bt.lookup_dev(dt.data_ptr(), len(master), dq.data_ptr(), len(has), out.data_ptr())
    torch.cuda.synchronize()
    assert [master[i][0] for i in out.cpu().tolist()] == [2, 3]
    img = c_tar_bytes()
    d = to_dev(torch, img)
    ok = torch.zeros(4, dtype=torch.uint8, device="cuda")
    bt.verify_dev(d.data_ptr(), 4, CHUNK, CHUNK, dt.data_ptr(), ok.data_ptr())
    torch.cuda.synchronize()
    assert name == "C.tar" and ok.cpu().tolist() == [1, 1, 1, 1]


def test_peer_download_flow_end_to_end(bt, torch, tmp_path):
    """The reference's integration oracle (p2-tests/tests.py:93-100: diff the
    downloaded file against the original) on the GPU path: the master .chunks
    file is parsed, the GET list is resolved with the GPU lookup (get_chunk_id,
    util.c:28-39), DATA payloads of 1484 bytes (common.h:30, network.c:301)
    arrive interleaved across chunks straight into verifier slots
    (save_data_packet, util.c:250-277), completed chunks are verified in
    batches (save_chunk, util.c:304-337; one corrupted transfer fails and is
    re-requested) and the verified slot bytes are written at id*512 KiB
    (util.c:322-325)."""
    import ctypes
    img = c_tar_bytes()
    name, master = bt.parse_master(os.path.join(GOLDEN, "ref_C.chunks"))
    get = bt.parse_chunk_list(os.path.join(GOLDEN, "ref_A.chunks")) + \
        bt.parse_chunk_list(os.path.join(GOLDEN, "ref_B.chunks"))
    dt = _dev_bytes(torch, b"".join(h for _, h in master))
    dq = _dev_bytes(torch, b"".join(h for _, h in get))
    idx = torch.zeros(len(get), dtype=torch.int64, device="cuda")
    bt.lookup_dev(dt.data_ptr(), len(master), dq.data_ptr(), len(get), idx.data_ptr())
    torch.cuda.synchronize()
    ids = [master[i][0] for i in idx.cpu().tolist()]
    assert name == "C.tar" and ids == [0, 1, 2, 3]
    expect = {cid: master[i][1] for cid, i in zip(ids, idx.cpu().tolist())}
    out = tmp_path / "out.tar"
    out.write_bytes(bytes(len(img)))
    v = bt.Verifier(batch=2, nstreams=2)
    rng = random.Random(3)
    received = {cid: 0 for cid in ids}
    slots = {cid: v.slot() for cid in ids}
    corrupt_next = {2}
    done, failures = set(), 0
    for _ in range(100000):
        if len(done) == len(ids):
            break
        for cid in ids:
            if cid in done or received[cid] == CHUNK or rng.random() < 0.5:
                continue
            off = received[cid]
            n = min(1484, CHUNK - off)
            data = img[cid * CHUNK + off:cid * CHUNK + off + n]
            if cid in corrupt_next and off == 0:
                data = bytes([data[0] ^ 1]) + data[1:]
            ctypes.memmove(slots[cid] + off, data, n)
            received[cid] = off + n
            if received[cid] == CHUNK:
                v.commit(slots[cid], expect[cid], tag=cid)
        verdicts = v.poll()
        if all(received[c] == CHUNK for c in ids if c not in done):
            verdicts += v.drain()
        for tag, ok, _ in verdicts:
            if ok:
                with open(out, "r+b") as f:
                    f.seek(tag * CHUNK)
                    f.write(ctypes.string_at(slots[tag], CHUNK))
                done.add(tag)
            else:  # util.c:317-319: "Verification failed!", chunk back to NOT_STARTED
                failures += 1
                corrupt_next.discard(tag)
                received[tag] = 0
                slots[tag] = v.slot()
    v.close()
    assert failures == 1
    assert out.read_bytes() == img  # diff A.tar test1.tar


def test_randomized_layouts_vs_oracle(bt, torch, oracle, rmode):
    """Seeded random batches: chunk length, pitch, count, input offset (alignment)
    and digest-output offset drawn at random, so both the hot kernel (aligned
    layouts) and the generic kernel (anything else) see shapes no fixed case
    names.  Every digest checked against the oracle."""
    rng = random.Random(0xB17)
    for case in range(40):
        chunk_len = rng.choice([rng.randrange(0, 200), rng.randrange(0, 5000), rng.randrange(60000, 70000)])
        pitch = chunk_len + rng.choice([0, 0, 16 - (chunk_len % 16 or 16), rng.randrange(0, 300)])
        pitch = max(pitch, 1)
        n = rng.choice([1, 2, 63, 64, 65, rng.randrange(1, 300)])
        in_off = rng.choice([0, 0, 16, rng.randrange(0, 16)])
        out_off = rng.choice([0, 0, 4, rng.randrange(0, 4)])
        total = pitch * (n - 1) + chunk_len
        host = bytearray(oracle.fill_synthetic(total + 16, case, 0xFEED))[:total]
        d = to_dev(torch, bytes(in_off) + bytes(host), pad=16)
        out = torch.zeros(20 * n + 8, dtype=torch.uint8, device="cuda")
        bt.chunks_dev(d.data_ptr() + in_off, n, chunk_len, pitch, out.data_ptr() + out_off)
        torch.cuda.synchronize()
        raw = bytes(out.cpu().numpy().tobytes())[out_off:out_off + 20 * n]
        for i in range(n):
            want = oracle.sha1(bytes(host[i * pitch:i * pitch + chunk_len]))
            assert raw[20 * i:20 * i + 20] == want, (case, chunk_len, pitch, n, in_off, out_off, i)


# ---- multi-device split on one GPU (bt_sha1_chunks_host_devices) ------------------
@pytest.mark.parametrize("workers", [2, 3, 8])
def test_multi_device_split_with_repeated_device_ids(bt, oracle, workers):
    """The multi-GPU host split (worker g takes chunks
    [g*n/G, (g+1)*n/G), one host thread, streams and staging lanes per worker,
    digests gathered in chunk order) run with `workers` workers on device 0.
    Checked against the reference's make-chunks output for C.tar (4 full
    chunks) and for the short-tail file (3 full chunks + 12345 B: the short
    chunk lands on the last worker)."""
    devs = [0] * workers
    img = c_tar_bytes()
    want_c = open(os.path.join(GOLDEN, "C.tar.make-chunks.out")).read()
    got = bt.chunks_host(img, devs=devs)
    assert "".join(f"{i} {d.hex()}\n" for i, d in enumerate(got)) == want_c
    tail = bytes(oracle.fill_synthetic(3 * CHUNK + 12345, 0, oracle.SEED_TAIL))
    want_t = open(os.path.join(GOLDEN, "tail.make-chunks.out")).read()
    got = bt.chunks_host(tail, devs=devs)
    assert "".join(f"{i} {d.hex()}\n" for i, d in enumerate(got)) == want_t
    # more chunks than one batch per worker, small chunks, short last chunk
    big = bytes(oracle.fill_synthetic(3 * 1024 * 1024 + 4097, 5, 11))
    assert bt.chunks_host(big, chunk_len=4096, devs=devs) == oracle.hash_chunks(big, 4096)
    # registered (pinned) image: every worker DMAs its own slice directly
    import numpy as np
    arr = np.frombuffer(bytearray(tail), dtype=np.uint8)
    bt.host_register(arr.ctypes.data, arr.nbytes)
    try:
        raw = bt.chunks_host_addr(arr.ctypes.data, arr.nbytes, devs=devs)
    finally:
        bt.host_unregister(arr.ctypes.data)
    assert "".join(f"{i} {raw[20 * i:20 * i + 20].hex()}\n" for i in range(len(raw) // 20)) == want_t


def test_multi_device_split_rejects_bad_lists(bt):
    with pytest.raises(bt.BtSha1Error, match="out of range"):
        bt.chunks_host(b"x" * 100, 64, devs=[0, 99])
    with pytest.raises(bt.BtSha1Error, match="empty"):
        bt.chunks_host(b"x" * 100, 64, devs=[])


# ---- NULL stream = the caller's default stream --------------------------
def test_null_stream_orders_after_default_stream_work(bt, torch, oracle):
    """A device call with stream=None must see input written by the caller's
    earlier default-stream kernels and must not race the caller's zeroing of
    the output: torch's default stream has handle 0, and NULL means exactly
    that stream.  The input is written at the end of a long default-stream
    queue (a chain of matmuls), so an unordered launch would read zeros."""
    assert torch.cuda.current_stream().cuda_stream == 0
    n = 256
    want = [bytes.fromhex(l.split()[1]) for l in open(os.path.join(GOLDEN, "synth4096.txt"))
            if not l.startswith("#")][:n]
    src = torch.empty(n * CHUNK, dtype=torch.uint8, device="cuda")
    bt.fill_synthetic(src.data_ptr(), n * CHUNK, 0, oracle.SEED_SYNTH, None)
    torch.cuda.synchronize()
    for trial in range(3):
        buf = torch.zeros(n * CHUNK, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        a = torch.randn(4096, 4096, device="cuda")
        for _ in range(20):  # ~tens of ms of default-stream work ahead of the copy
            a = a @ a
            a = a / (a.abs().max() + 1)
        buf.copy_(src)  # written only after the matmul chain
        dig = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
        bt.chunks_dev(buf.data_ptr(), n, CHUNK, CHUNK, dig.data_ptr(), None)
        dig2 = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
        bt.fill_synthetic(dig2.data_ptr(), 16, 0, 1, None)  # a NULL-stream write the caller then overwrites
        dig2.zero_()
        torch.cuda.synchronize()
        assert digests_of(torch, dig, n) == want, trial
        assert int(dig2.sum().item()) == 0, trial


def test_kernel_name_reports_the_launch(bt, torch):
    """Default thresholds follow the device's CU count (256 on a full MI355X):
    chain kernel up to 2 chunks per CU, latency kernel up to 128 per CU."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    lat = bt.set_latency_batch(2**64 - 1)  # auto
    chain = bt.set_chain_batch(2**64 - 1)
    try:
        assert bt.kernel_name(1) == "k_sha1_chain"
        assert bt.kernel_name(2 * cus) == "k_sha1_chain"
        assert bt.kernel_name(2 * cus + 1) == "k_sha1_lat"
        assert bt.kernel_name(128 * cus) == "k_sha1_lat"
        assert bt.kernel_name(128 * cus + 1) == "k_sha1_fixed"
        assert bt.kernel_name(131072) == ("k_sha1_fixed" if 128 * cus < 131072 else "k_sha1_lat")
        assert "latency_batch=auto" in bt.build_info()
    finally:
        bt.set_latency_batch(lat)
        bt.set_chain_batch(chain)


def test_clock_probe_stamps_and_digests(bt, torch, oracle):
    """The bench's clock probe hashes exactly like the production kernel and
    leaves one sane stamp quadruple per wave."""
    n = 4096
    buf = torch.empty(n * CHUNK, dtype=torch.uint8, device="cuda")
    bt.fill_synthetic(buf.data_ptr(), n * CHUNK, 0, oracle.SEED_SYNTH, None)
    dig = torch.zeros(20 * n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(4 * (n // 64), dtype=torch.int64, device="cuda")
    bt.clock_probe(buf.data_ptr(), n, CHUNK, CHUNK, dig.data_ptr(), st.data_ptr(), None)
    torch.cuda.synchronize()
    want = [bytes.fromhex(l.split()[1]) for l in open(os.path.join(GOLDEN, "synth4096.txt"))
            if not l.startswith("#")]
    assert digests_of(torch, dig, n) == want
    s = st.view(-1, 4).cpu()
    dm, dr = (s[:, 2] - s[:, 0]).double(), (s[:, 3] - s[:, 1]).double()
    assert bool((dm > 0).all()) and bool((dr > 0).all())
    mhz = float((dm / dr).median()) * bt.wallclock_khz() / 1000.0
    assert 500.0 < mhz < 3000.0, mhz


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 129, 200])
def test_chain_kernel_many_blocks_and_batches(bt, torch, oracle, n):
    """Chain kernel batch boundaries: messages whose block counts straddle the
    loader wave's 64-block batches (and the two LDS slots), with every
    padding residue, against the oracle."""
    with ragged_mode(bt, "chain"):
        lens = [64 * n + r for r in (0, 1, 55, 56, 63)] + [64 * n - 8, 64 * 64 * 2 + n]
        blob = bytes(oracle.fill_synthetic(sum(lens) + 64, n, 0xC4A1))
        offs, o = [], 0
        for L in lens:
            offs.append(o)
            o += L
        d = to_dev(torch, blob)
        ot = torch.tensor(offs, dtype=torch.int64, device="cuda")
        lt = torch.tensor(lens, dtype=torch.int32, device="cuda")
        out = torch.zeros(20 * len(lens) + 3, dtype=torch.uint8, device="cuda")
        bt.ragged_dev(d.data_ptr(), ot.data_ptr(), lt.data_ptr(), len(lens), out.data_ptr() + 3)
        torch.cuda.synchronize()
        raw = bytes(out.cpu().numpy().tobytes())[3:]
        for i, (off, L) in enumerate(zip(offs, lens)):
            assert raw[20 * i:20 * i + 20] == oracle.sha1(blob[off:off + L]), (n, L)


def test_streaming_update_pieces_and_context(bt, oracle):
    """SHA1Update through the chain kernel's midstate mode, fed the way the
    peer receives a chunk (1484-byte DATA payloads, util.c:275) and in odd
    pieces, with SHA1Context.hash / totalLength / bufferLength checked after
    every call against the oracle's own streaming context."""
    msg = bytes(oracle.fill_synthetic(CHUNK, 0, oracle.SEED_SYNTH))
    s = bt.Sha1()
    o = oracle.Sha1Stream()
    i, k = 0, 0
    pieces = [1484, 1, 63, 64, 65, 4096, 1484 * 7, 100000]
    while i < len(msg):
        j = min(len(msg), i + pieces[k % len(pieces)])
        s.update(msg[i:j])
        o.update(msg[i:j])
        k += 1
        i = j
        assert s.ctx.totalLength == 8 * i and s.ctx.bufferLength == i % 64
        if k % 17 == 0:
            done = i - i % 64
            assert list(s.ctx.hash) == oracle.compress_blocks(
                [0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476, 0xc3d2e1f0], msg[:done]), k
    assert s.final() == o.final() == oracle.sha1(msg)


def test_streaming_context_equals_the_reference_context(bt, oracle):
    """The drop-in's SHA1Context against the REFERENCE's own (sha.c's
    SHA1Init / SHA1Update / SHA1Final, compiled into oracle/_ref/libref_sha1.so,
    same 96-byte layout, sha.h:39-50): after every SHA1Update of random length
    (0..5000 bytes, so calls end at every offset within a block and some carry
    no whole block) the two contexts agree on totalLength, hash[5],
    bufferLength and the buffered bytes; the digests agree at the end."""
    ref_path = os.path.join(REPO, "oracle", "_ref", "libref_sha1.so")
    assert os.path.exists(ref_path), "oracle/_ref/libref_sha1.so missing: built by oracle/Makefile"
    ref = ctypes.CDLL(ref_path)
    ctx_t = bt.SHA1Context
    ref.SHA1Init.argtypes = [ctypes.POINTER(ctx_t)]
    ref.SHA1Update.argtypes = [ctypes.POINTER(ctx_t), ctypes.c_void_p, ctypes.c_uint32]
    ref.SHA1Final.argtypes = [ctypes.POINTER(ctx_t), ctypes.c_void_p]
    rng = random.Random(4242)
    for trial in range(3):
        msg = bytes(oracle.fill_synthetic(150000 + trial * 7919, trial, 0x5EED))
        rc = ctx_t()
        ref.SHA1Init(ctypes.byref(rc))
        s = bt.Sha1()
        i = calls = 0
        while i < len(msg):
            j = min(len(msg), i + rng.choice([0, 1, 55, 56, 63, 64, 65, rng.randrange(5000)]))
            piece = msg[i:j]
            buf = (ctypes.c_uint8 * max(1, len(piece))).from_buffer_copy(piece or b"\0")
            ref.SHA1Update(ctypes.byref(rc), buf, len(piece))
            s.update(piece)
            i, calls = j, calls + 1
            n = rc.bufferLength
            assert (s.ctx.totalLength, list(s.ctx.hash), s.ctx.bufferLength) == \
                (rc.totalLength, list(rc.hash), n), (trial, calls, i)
            assert bytes(s.ctx.buffer[:n]) == bytes(rc.buffer[:n]), (trial, calls, i)
        out = (ctypes.c_uint8 * 20)()
        ref.SHA1Final(ctypes.byref(rc), out)
        assert s.final() == bytes(out) == oracle.sha1(msg), trial


def test_dropin_calls_from_many_threads(bt, oracle):
    """shahash / SHA1Update / SHA1Final from several host threads at once (the
    calls share one device context and its pinned staging; ctypes releases the
    GIL, so they really overlap) and two SHA1Context streams interleaved on
    one thread: every digest equals the oracle's."""
    import threading
    msgs = [bytes(oracle.fill_synthetic(n, 17 * n, 0x7E57)) for n in (0, 55, 64, 1000, 70000, CHUNK, CHUNK + 3)]
    want = [oracle.sha1(m) for m in msgs]
    errors = []

    def worker(k):
        try:
            for rep in range(3):
                for i, m in enumerate(msgs):
                    if (i + k + rep) % 2:
                        got = bt.shahash(m)
                    else:
                        s = bt.Sha1()
                        step = 1484 if len(m) > 4096 else 7
                        for o in range(0, len(m), step):
                            s.update(m[o:o + step])
                        got = s.final()
                    if got != want[i]:
                        errors.append((k, rep, i))
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]
    # two contexts interleaved
    a, b = bt.Sha1(), bt.Sha1()
    ma, mb = msgs[5], msgs[6]
    for o in range(0, max(len(ma), len(mb)), 4096):
        a.update(ma[o:o + 4096])
        b.update(mb[o:o + 4096])
    assert a.final() == want[5] and b.final() == want[6]



@pytest.mark.parametrize("n", [65, 600, 4099])
def test_ragged_latency_kernel_mixed_lengths(bt, torch, oracle, n):
    """k_sha1_lat_ragged: 64 messages per workgroup with unequal lengths (so
    lanes finish at different blocks and latch their own state), every
    residue mod 64 incl. messages shorter than one block (those lanes read a
    static zero block), odd offsets; and the launch past one workgroup per CU
    (three-slot form) at n = 4099.  Against the oracle."""
    rng = random.Random(n)
    lens = [rng.choice([0, 1, 55, 56, 63, 64, 65, 119, 120, 1000, rng.randrange(0, 40000)]) for _ in range(n)]
    offs, pos = [], 0
    for L in lens:
        pos += rng.randrange(0, 16)
        offs.append(pos)
        pos += L
    blob = bytes(oracle.fill_synthetic(pos + 64, n, 0x1A7))
    d = to_dev(torch, blob)
    ot = torch.tensor(offs, dtype=torch.int64, device="cuda")
    lt = torch.tensor(lens, dtype=torch.int32, device="cuda")
    out = torch.zeros(20 * n + 1, dtype=torch.uint8, device="cuda")
    with ragged_mode(bt, "latr"):
        bt.ragged_dev(d.data_ptr(), ot.data_ptr(), lt.data_ptr(), n, out.data_ptr() + 1)
        torch.cuda.synchronize()
    raw = bytes(out.cpu().numpy().tobytes())[1:]
    for i in range(n):
        assert raw[20 * i:20 * i + 20] == oracle.sha1(blob[offs[i]:offs[i] + lens[i]]), (n, i, lens[i])
