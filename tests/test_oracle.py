"""CPU: pin the oracle (our restatement) to the reference's golden vectors.

Every expected value comes from the reference itself: its fixture files
(p2-tests/*.chunks, copied as tests/golden/ref_*.chunks), its self-test KATs
(sha.c:32-38, chunk.c:86-104) and digests the compiled reference produced for
the committed inputs (tests/golden/make_golden.py).
"""
import hashlib
import os
import random

import numpy as np
import pytest

from conftest import c_tar_bytes, read_pairs, GOLDEN

CHUNK = 512 * 1024


def test_kats(oracle):
    data = {"abc": b"abc", "dash": b"dash", "empty": b"",
            "nist448": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
            "zeros_512k": bytes(CHUNK), "ff_512k": b"\xff" * CHUNK,
            "iota_512k": bytes(i & 255 for i in range(CHUNK)), "million_a": b"a" * 1000000}
    rows = read_pairs("kat.txt")
    assert len(rows) == 8
    for name, n, h in rows:
        assert len(data[name]) == int(n)
        assert oracle.sha1(data[name]).hex() == h, name


def test_sha_c_selftest_strings(oracle):
    # sha.c:35-37 (printed with spaces every 4 bytes by its SHA1_TEST main)
    assert oracle.sha1(b"abc").hex() == "a9993e364706816aba3e25717850c26c9cd0d89d"
    s = oracle.Sha1Stream()
    for _ in range(1000):
        s.update(b"a" * 1000)
    assert s.final().hex() == "34aa973cd4c4daa4f61eeb2bdbad27316534016f"


def test_c_tar_matches_reference_chunks_files(oracle):
    img = c_tar_bytes()
    assert len(img) == 4 * CHUNK
    got = [oracle.sha1(img[i * CHUNK:(i + 1) * CHUNK]).hex() for i in range(4)]
    # p2-tests/C.chunks:3-6 (after the "File:" / "Chunks:" header)
    ref_c = [tuple(l.split()) for l in open(f"{GOLDEN}/ref_C.chunks").read().splitlines()[2:]]
    assert [(str(i), h) for i, h in enumerate(got)] == ref_c
    # p2-tests/A.chunks = test1.chunks = chunks 0-1; B.chunks = chunks 2-3 with global ids
    assert read_pairs("ref_A.chunks") == [("0", got[0]), ("1", got[1])]
    assert read_pairs("ref_test1.chunks") == [("0", got[0]), ("1", got[1])]
    assert read_pairs("ref_B.chunks") == [("2", got[2]), ("3", got[3])]
    # make-chunks C.tar stdout, byte for byte
    lines = "".join(f"{i} {h}\n" for i, h in enumerate(got))
    assert open(f"{GOLDEN}/C.tar.make-chunks.out").read() == lines


def test_edge_lengths(oracle):
    rows = read_pairs("edge_lengths.txt")
    stream = bytes(oracle.fill_synthetic(max(int(n) for n, _ in rows), 0, oracle.SEED_EDGE))
    for n, h in rows:
        assert oracle.sha1(stream[:int(n)]).hex() == h, n


def test_ragged_golden(oracle):
    for k, n, h in read_pairs("ragged.txt"):
        k, n = int(k), int(n)
        assert n == oracle.ragged_len(k)
        assert oracle.sha1(bytes(oracle.fill_synthetic(n, k * 1024, oracle.SEED_RAGGED))).hex() == h


def test_tail_file_make_chunks_output(oracle):
    data = bytes(oracle.fill_synthetic(3 * CHUNK + 12345, 0, oracle.SEED_TAIL))
    dig = oracle.hash_chunks(data, CHUNK)
    assert len(dig) == 4
    out = "".join(f"{i} {d.hex()}\n" for i, d in enumerate(dig))
    assert open(f"{GOLDEN}/tail.make-chunks.out").read() == out


def test_synth4096_sample(oracle):
    rows = read_pairs("synth4096.txt")
    assert len(rows) == 4096
    pick = [0, 1, 2, 63, 64, 255, 256, 1023, 2048, 4031, 4095]
    for i in pick:
        data = bytes(oracle.fill_synthetic(CHUNK, i * (CHUNK // 8), oracle.SEED_SYNTH))
        assert rows[i] == (str(i), oracle.sha1(data).hex())


def test_synth_digests_equal_every_golden_row(oracle):
    """The bulk sweep the GPU tests check whole batches with (each chunk
    regenerated in C, threaded) reproduces ALL 4096 digests the compiled
    reference produced (tests/golden/synth4096.txt), and equals hashing the
    generated image for other chunk sizes and first chunks."""
    rows = read_pairs("synth4096.txt")
    d = oracle.synth_digests(0, 4096)
    assert [(str(i), d[20 * i:20 * i + 20].hex()) for i in range(4096)] == rows
    img = oracle.fill_synthetic(9 * 4096, 1000 * 512, 31)
    assert oracle.synth_digests(1000, 9, 4096, 31, nthreads=3) == b"".join(oracle.hash_chunks(img, 4096))
    with pytest.raises(ValueError):
        oracle.synth_digests(0, 1, 12)


def test_batch_checksums_are_the_reference_digests(oracle):
    """tests/golden/synth_checksums.txt (the reference's digests of the bench's
    synthetic chunks, checksummed per global chunk count): its 4096 row agrees
    with the 4096 golden digests, and the oracle's sweep reproduces the
    smaller rows; the config-4 row (1,048,576 chunks) is what bench.py's
    parity_all_vs_golden compares an 8-GPU run with."""
    table = dict(read_pairs("synth_checksums.txt"))
    assert {"4096", "81920", "131072", "262144", "327680", "524288", "1048576"} <= set(table)
    rows = read_pairs("synth4096.txt")
    assert hashlib.sha1(b"".join(bytes.fromhex(h) for _, h in rows)).hexdigest() == table["4096"]
    assert hashlib.sha1(oracle.synth_digests(0, 81920)).hexdigest() == table["81920"]


def test_generator_matches_numpy_splitmix(oracle):
    """The frozen generator (shared with the device kernel) restated in numpy."""
    def splitmix(x):
        with np.errstate(over="ignore"):
            z = x + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            return z ^ (z >> np.uint64(31))
    first, seed = 123456789, oracle.SEED_SYNTH
    g = np.arange(first, first + 1000, dtype=np.uint64)
    want = splitmix(np.uint64(seed) + g).astype("<u8").tobytes()
    assert bytes(oracle.fill_synthetic(8000, first, seed)) == want
    assert bytes(oracle.fill_synthetic(8003, first, seed))[:8000] == want  # ragged tail
    # wrap-around of seed + word index is modulo 2^64
    big = np.uint64(2**64 - 5)
    assert bytes(oracle.fill_synthetic(80, 0, 2**64 - 5)) == splitmix(big + np.arange(10, dtype=np.uint64)).astype("<u8").tobytes()


def test_streaming_splits_match_one_shot(oracle):
    rng = random.Random(7)
    for trial in range(40):
        n = rng.choice([0, 1, 63, 64, 65, 200, 4097, 70000])
        data = rng.randbytes(n)
        s = oracle.Sha1Stream()
        i = 0
        while i < n:
            j = min(n, i + rng.choice([1, 7, 63, 64, 65, 1000]))
            s.update(data[i:j])
            i = j
        d = s.final()
        assert d == oracle.sha1(data) == hashlib.sha1(data).digest()


def test_hex_codec(oracle):
    b = bytes(range(0, 256, 13))[:20]
    h = oracle.binary2hex(b)
    assert h == b.hex() and oracle.hex2binary(h) == b
    assert oracle.hex2binary(h.upper()) == b
    # chunk.c:66-71 accepts non-hex silently: 'g' -> 'G' - ('A' - 10) = 16
    assert oracle.hex2binary("0g") == bytes([16])


def test_threaded_batch_equals_serial(oracle):
    data = bytearray(oracle.fill_synthetic(9 * 4096 + 100, 5, 99))
    a = oracle.hash_chunks(data, 4096, nthreads=1)
    b = oracle.hash_chunks(data, 4096, nthreads=4)
    assert a == b and len(a) == 10
    assert a[-1] == hashlib.sha1(bytes(data[9 * 4096:])).digest()


def test_reference_library_agrees_when_built(oracle):
    ref = oracle.load_reference()
    if ref is None:
        pytest.skip("oracle/_ref not built (reference absent)")
    import ctypes
    for n in [0, 1, 55, 56, 64, 1000, CHUNK]:
        d = bytes(oracle.fill_synthetic(n, 3, 4))
        out = (ctypes.c_uint8 * 20)()
        ref.shahash((ctypes.c_uint8 * max(n, 1)).from_buffer_copy(d or b"\0"), n, out)
        assert bytes(out) == oracle.sha1(d)


def test_oracle_under_asan_ubsan(tmp_path):
    """Host-code sanitizers on the restatement (GPU sanitizers are not available)."""
    import subprocess
    from conftest import REPO
    exe = tmp_path / "oracle_asan"
    src = [f"{REPO}/oracle/sha1_oracle.c", f"{REPO}/oracle/oracle_selftest.c"]
    r = subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-fno-omit-frame-pointer", "-pthread", "-o", str(exe)] + src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env)
    assert r.returncode == 0 and "ok (0 failures)" in r.stdout, r.stdout + r.stderr


def test_batch_drivers_report_refused_threads_cleanly():
    """or_hash_chunks / or_synth_digests (the parity checker's threaded sweeps)
    with more threads than RLIMIT_NPROC allows, in a child process run as an
    unprivileged user: -1 (every started thread joined, none of the unset
    handles), not a crash and not a 0 over a partly written output."""
    import subprocess
    import sys
    from conftest import REPO
    code = r'''
import ctypes, os, resource, sys
lib = ctypes.CDLL(sys.argv[1])
vp, u64 = ctypes.c_void_p, ctypes.c_uint64
lib.or_synth_digests.argtypes = [u64, u64, ctypes.c_uint32, u64, vp, ctypes.c_int]
lib.or_hash_chunks.argtypes = [vp, u64, u64, ctypes.c_uint32, ctypes.c_uint32, vp, ctypes.c_int]
n, L = 64, 4096
img = (ctypes.c_uint8 * (n * L))()
out = (ctypes.c_uint8 * (20 * n))()
ok_all = lib.or_synth_digests(0, n, L, 77, out, 8)       # unrestricted: 0
try:
    if os.geteuid() == 0:
        os.setgid(65534)
        os.setuid(65534)
    resource.setrlimit(resource.RLIMIT_NPROC, (1, 1))
except OSError as e:  # uid 65534 unmapped / setuid not permitted: the limit would not bind
    print("SKIP", e)
    sys.exit(0)
print(ok_all, lib.or_synth_digests(0, n, L, 77, out, 8), lib.or_hash_chunks(img, n, L, L, L, out, 16))
'''
    r = subprocess.run([sys.executable, "-c", code, f"{REPO}/oracle/liboracle_sha1.so"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    if r.stdout.startswith("SKIP"):
        pytest.skip(f"cannot drop to an unprivileged user here: {r.stdout.strip()}")
    assert r.stdout.split() == ["0", "-1", "-1"], r.stdout
