"""btsha1 -- ctypes binding of libbtsha1.so (the C-ABI in include/bt_sha1.h).

This is the binding a Python caller (tests, bench.py) uses; C callers link the
library directly.  Device buffers are passed as raw integer
addresses (e.g. ``tensor.data_ptr()``) and streams as raw ``hipStream_t``
handles (``torch.cuda.current_stream().cuda_stream``), so nothing here depends
on torch.  There is no fallback: if the library cannot be loaded, importing
this module raises, and every call that fails on the GPU raises BtSha1Error
with the library's own message.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BT_SHA1_LIB", os.path.join(HERE, "libbtsha1.so"))
CHUNK = 512 * 1024  # BT_CHUNK_SIZE, chunk.h:16
DIGEST = 20  # SHA1_HASH_SIZE, sha.h:34


class BtSha1Error(RuntimeError):
    pass


if not os.path.exists(LIB_PATH):
    raise ImportError(f"libbtsha1.so not built at {LIB_PATH}: run `make` (or __graft_entry__.build())")
lib = ctypes.CDLL(LIB_PATH)

_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_i64 = ctypes.c_int64


class Verdict(ctypes.Structure):
    _fields_ = [("tag", ctypes.c_uint64), ("ok", ctypes.c_int32), ("digest", ctypes.c_uint8 * 20)]


class SHA1Context(ctypes.Structure):  # include/sha.h (reference sha.h:39-50 layout)
    _fields_ = [("totalLength", ctypes.c_uint64), ("hash", ctypes.c_uint32 * 5),
                ("bufferLength", ctypes.c_uint32), ("buffer", ctypes.c_uint8 * 64)]


STATS_NODES = 8  # BT_SHA1_STATS_NODES


class PipelineStats(ctypes.Structure):  # include/bt_sha1.h bt_sha1_pipeline_stats
    _fields_ = [("chunks", ctypes.c_uint64), ("bytes", ctypes.c_uint64), ("batch_bytes", ctypes.c_uint64),
                ("batches", ctypes.c_uint32), ("staged", ctypes.c_int32), ("device", ctypes.c_int32),
                ("copy_threads", ctypes.c_int32), ("numa_nodes", ctypes.c_int32),
                ("gpu_numa_node", ctypes.c_int32), ("numa_policy", ctypes.c_int32),
                ("registered_batches", ctypes.c_int32), ("column_chunks", ctypes.c_uint32),
                ("total_s", ctypes.c_double), ("alloc_s", ctypes.c_double), ("fill_s", ctypes.c_double),
                ("wait_s", ctypes.c_double), ("register_s", ctypes.c_double), ("unregister_s", ctypes.c_double),
                ("lane_pages", ctypes.c_int32 * STATS_NODES), ("src_pages", ctypes.c_int32 * STATS_NODES),
                ("copy_pieces", ctypes.c_int32 * STATS_NODES)]


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("bt_sha1_device_count", ctypes.c_int)
_sig("bt_sha1_set_device", ctypes.c_int, ctypes.c_int)
_sig("bt_sha1_last_error", ctypes.c_char_p)
_sig("bt_sha1_build_info", ctypes.c_char_p)
_sig("bt_sha1_set_ring_depth", ctypes.c_int, ctypes.c_int)
_sig("bt_sha1_set_variant", ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int)
_sig("bt_sha1_set_latency_batch", _u64, _u64)
_sig("bt_sha1_chunks_dev", ctypes.c_int, _vp, _u64, _u64, _u64, _vp, _vp)
_sig("bt_sha1_verify_dev", ctypes.c_int, _vp, _u64, _u64, _u64, _vp, _vp, _vp, _vp)
_sig("bt_sha1_ragged_dev", ctypes.c_int, _vp, _vp, _vp, _u64, _vp, _vp)
_sig("bt_sha1_fill_synthetic", ctypes.c_int, _vp, _u64, _u64, _u64, _vp)
_sig("bt_sha1_chunks_host", _i64, _vp, _u64, _u64, _vp)
_sig("bt_sha1_host_register", ctypes.c_int, _vp, _u64)
_sig("bt_sha1_host_unregister", ctypes.c_int, _vp)
_sig("bt_sha1_chunks_host_multi", _i64, _vp, _u64, _u64, _vp, ctypes.c_int)
_sig("bt_sha1_chunks_host_devices", _i64, _vp, _u64, _u64, _vp, ctypes.POINTER(ctypes.c_int), ctypes.c_int)
_sig("bt_sha1_source_id", ctypes.c_char_p)
_sig("bt_sha1_set_chain_batch", _u64, _u64)
_sig("bt_sha1_kernel_name", ctypes.c_char_p, _u64)
_sig("bt_sha1_clock_probe", ctypes.c_int, _vp, _u64, _u64, _u64, _vp, _vp, _vp)
_sig("bt_sha1_wallclock_khz", _i64)
_sig("bt_sha1_debug_barrier_stats", ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int)
_sig("bt_sha1_debug_dropin_residue", _i64, ctypes.c_int)
_sig("bt_sha1_chunks_file", _i64, _vp, _u64, _vp, _u64)
_sig("bt_sha1_get_pipeline_stats", ctypes.c_int, ctypes.POINTER(PipelineStats))
_sig("bt_sha1_set_pageable_feed", ctypes.c_int, ctypes.c_int)
_sig("bt_sha1_verifier_create", _vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32)
_sig("bt_sha1_verifier_destroy", None, _vp)
_sig("bt_sha1_verifier_slot", _vp, _vp)
_sig("bt_sha1_verifier_commit", ctypes.c_int, _vp, _vp, ctypes.c_uint32, _vp, _u64)
_sig("bt_sha1_verifier_release", ctypes.c_int, _vp, _vp)
_sig("bt_sha1_verifier_submit", ctypes.c_int, _vp, _vp, ctypes.c_uint32, _vp, _u64)
_sig("bt_sha1_verifier_flush", ctypes.c_int, _vp)
_sig("bt_sha1_verifier_poll", ctypes.c_int, _vp, ctypes.POINTER(Verdict), ctypes.c_int)
_sig("bt_sha1_verifier_drain", ctypes.c_int, _vp, ctypes.POINTER(Verdict), ctypes.c_int)
_sig("bt_sha1_verifier_pending", _i64, _vp)
_sig("bt_sha1_lookup_dev", ctypes.c_int, _vp, _u64, _vp, _u64, _vp, _vp)


class ChunkEntry(ctypes.Structure):
    _fields_ = [("id", ctypes.c_int32), ("hash", ctypes.c_uint8 * 20)]


_sig("bt_chunks_parse_list", _i64, ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(ChunkEntry)))
_sig("bt_chunks_parse_master", _i64, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
     ctypes.POINTER(ctypes.POINTER(ChunkEntry)))
_sig("bt_chunks_free", None, ctypes.POINTER(ChunkEntry))
_sig("bt_chunks_write", ctypes.c_int, _vp, ctypes.c_char_p, _vp, ctypes.c_int64, ctypes.c_int32)
_sig("bt_hex2binary_checked", ctypes.c_int, ctypes.c_char_p, ctypes.c_int, _vp)
_sig("bt_chunks_last_error", ctypes.c_char_p)
_sig("SHA1Init", None, ctypes.POINTER(SHA1Context))
_sig("SHA1Update", None, ctypes.POINTER(SHA1Context), _vp, ctypes.c_uint32)
_sig("SHA1Final", None, ctypes.POINTER(SHA1Context), _vp)
_sig("shahash", None, _vp, ctypes.c_int, _vp)
_sig("binary2hex", None, _vp, ctypes.c_int, ctypes.c_char_p)
_sig("hex2binary", None, ctypes.c_char_p, ctypes.c_int, _vp)


def _check(rc, what):
    if rc is None or (isinstance(rc, int) and rc < 0):
        raise BtSha1Error(f"{what}: {lib.bt_sha1_last_error().decode()}")
    return rc


def last_error():
    return lib.bt_sha1_last_error().decode()


def device_count():
    return lib.bt_sha1_device_count()


def set_ring_depth(nbuf):
    _check(lib.bt_sha1_set_ring_depth(nbuf), "set_ring_depth")


def set_variant(nbuf, lines=1, nt=0):
    _check(lib.bt_sha1_set_variant(nbuf, lines, nt), "set_variant")


def set_latency_batch(max_chunks):
    """Batches of <= max_chunks take the latency kernel (0: never); returns the previous value."""
    return lib.bt_sha1_set_latency_batch(max_chunks)


def set_chain_batch(max_messages):
    """Ragged batches of <= max_messages take the chain kernel (0: never); returns the previous setting."""
    return lib.bt_sha1_set_chain_batch(max_messages)


def build_info():
    return lib.bt_sha1_build_info().decode()


def source_id():
    """Id of the kernel sources compiled into the library (profiles record it)."""
    return lib.bt_sha1_source_id().decode()


def kernel_name(n_chunks):
    """Kernel a fixed-layout batch of n_chunks runs on the current device."""
    r = lib.bt_sha1_kernel_name(n_chunks)
    if r is None:
        raise BtSha1Error(f"bt_sha1_kernel_name: {last_error()}")
    return r.decode()


def clock_probe(d_in, n, chunk_len, pitch, d_digests, d_stamps, stream=None):
    """Stamped diagnostic build of the hot kernel (4 uint64 per wave into d_stamps)."""
    _check(lib.bt_sha1_clock_probe(d_in, n, chunk_len, pitch, d_digests, d_stamps, stream), "bt_sha1_clock_probe")


def wallclock_khz():
    return _check(lib.bt_sha1_wallclock_khz(), "bt_sha1_wallclock_khz")


def debug_barrier_stats(reset=False):
    """(waves checked, barriers executed, invariant misses) of the barrier-
    accounting build (make dbgbar, loaded with BT_SHA1_LIB); raises on the
    production library, which counts nothing."""
    out = (ctypes.c_uint64 * 3)()
    _check(lib.bt_sha1_debug_barrier_stats(out, 1 if reset else 0), "bt_sha1_debug_barrier_stats")
    return tuple(int(x) for x in out)


def debug_dropin_residue(device=0):
    """Nonzero bytes left in the drop-in calls' pinned staging on `device`
    (0 between calls: each shahash / SHA1Update / SHA1Final zeroes what it
    staged, as chunk.c:48 and sha.c:165-174 leave nothing behind)."""
    return _check(lib.bt_sha1_debug_dropin_residue(device), "bt_sha1_debug_dropin_residue")


# ---- device-resident (addresses are ints) ------------------------------------
def chunks_dev(d_in, n, chunk_len, pitch, d_digests, stream=None):
    _check(lib.bt_sha1_chunks_dev(d_in, n, chunk_len, pitch, d_digests, stream), "bt_sha1_chunks_dev")


def verify_dev(d_in, n, chunk_len, pitch, d_expected, d_ok, d_digests=None, stream=None):
    _check(lib.bt_sha1_verify_dev(d_in, n, chunk_len, pitch, d_expected, d_ok, d_digests, stream),
           "bt_sha1_verify_dev")


def ragged_dev(d_base, d_offsets, d_lens, n, d_digests, stream=None):
    _check(lib.bt_sha1_ragged_dev(d_base, d_offsets, d_lens, n, d_digests, stream), "bt_sha1_ragged_dev")


def fill_synthetic(d_buf, nbytes, first_word, seed, stream=None):
    _check(lib.bt_sha1_fill_synthetic(d_buf, nbytes, first_word, seed, stream), "bt_sha1_fill_synthetic")


def lookup_dev(d_table, n_table, d_queries, n_queries, d_index, stream=None):
    _check(lib.bt_sha1_lookup_dev(d_table, n_table, d_queries, n_queries, d_index, stream), "bt_sha1_lookup_dev")


# ---- .chunks files (host-side parsing/formatting) ---------------------------------
def _entries(ptr, n):
    try:
        return [(ptr[i].id, bytes(ptr[i].hash)) for i in range(n)]
    finally:
        lib.bt_chunks_free(ptr)


def parse_chunk_list(path):
    """[(id, digest)] of a has/get .chunks file (util.c:64-111)."""
    p = ctypes.POINTER(ChunkEntry)()
    n = lib.bt_chunks_parse_list(str(path).encode(), ctypes.byref(p))
    if n < 0:
        raise BtSha1Error(lib.bt_chunks_last_error().decode())
    return _entries(p, n)


def parse_master(path):
    """(data file name, [(id, digest)]) of a master .chunks file (util.c:113-164)."""
    p = ctypes.POINTER(ChunkEntry)()
    name = ctypes.create_string_buffer(1024)
    n = lib.bt_chunks_parse_master(str(path).encode(), name, 1024, ctypes.byref(p))
    if n < 0:
        raise BtSha1Error(lib.bt_chunks_last_error().decode())
    return name.value.decode(), _entries(p, n)


def write_chunks(path, digests, master_name=None, first_id=0):
    libc = ctypes.CDLL(None)
    libc.fopen.restype = _vp
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [_vp]
    raw = b"".join(digests)
    fp = libc.fopen(str(path).encode(), b"w")
    try:
        buf = (ctypes.c_uint8 * max(len(raw), 1)).from_buffer_copy(raw or b"\0")
        rc = lib.bt_chunks_write(fp, master_name.encode() if master_name else None, buf, len(digests), first_id)
    finally:
        libc.fclose(fp)
    if rc:
        raise BtSha1Error(lib.bt_chunks_last_error().decode())


def hex2binary_checked(h):
    hb = h.encode() if isinstance(h, str) else bytes(h)
    out = (ctypes.c_uint8 * max(len(hb) // 2, 1))()
    if lib.bt_hex2binary_checked(hb, len(hb), out):
        raise ValueError(f"not hex: {h!r}")
    return bytes(out)[:len(hb) // 2]


# ---- host ------------------------------------------------------------------------
def _host_buf(data):
    if isinstance(data, (bytes, bytearray)):
        b = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(bytes(data) or b"\0")
        return b, len(data)
    mv = memoryview(data).cast("B")
    arr = (ctypes.c_uint8 * max(mv.nbytes, 1)).from_buffer(mv) if not mv.readonly else \
        (ctypes.c_uint8 * max(mv.nbytes, 1)).from_buffer_copy(mv.tobytes() or b"\0")
    return arr, mv.nbytes


def _host_split(addr, nbytes, chunk_len, out, ndev, devs):
    if devs is not None:
        arr = (ctypes.c_int * max(len(devs), 1))(*devs)
        return _check(lib.bt_sha1_chunks_host_devices(addr, nbytes, chunk_len, out, arr, len(devs)),
                      "bt_sha1_chunks_host_devices")
    if ndev is not None:
        return _check(lib.bt_sha1_chunks_host_multi(addr, nbytes, chunk_len, out, ndev), "bt_sha1_chunks_host_multi")
    return _check(lib.bt_sha1_chunks_host(addr, nbytes, chunk_len, out), "bt_sha1_chunks_host")


def chunks_host(data, chunk_len=CHUNK, ndev=None, devs=None):
    """Digests of data cut into chunk_len pieces (short last piece): list of 20-byte values.
    ndev: split over the first ndev GPUs; devs: split over this list of device
    ids (repeats allowed: one worker per entry)."""
    buf, n = _host_buf(data)
    nch = (n + chunk_len - 1) // chunk_len
    out = (ctypes.c_uint8 * max(20 * nch, 1))()
    got = _host_split(buf, n, chunk_len, out, ndev, devs)
    raw = bytes(out)
    return [raw[20 * i:20 * i + 20] for i in range(got)]


def host_register(addr, nbytes):
    """Page-lock host memory at integer address `addr` (DMA without staging)."""
    _check(lib.bt_sha1_host_register(addr, nbytes), "bt_sha1_host_register")


def host_unregister(addr):
    _check(lib.bt_sha1_host_unregister(addr), "bt_sha1_host_unregister")


def chunks_host_addr(addr, nbytes, chunk_len=CHUNK, ndev=None, devs=None):
    """bt_sha1_chunks_host over raw host memory at `addr` (no copy on the Python side)."""
    nch = (nbytes + chunk_len - 1) // chunk_len
    out = (ctypes.c_uint8 * max(20 * nch, 1))()
    got = _host_split(addr, nbytes, chunk_len, out, ndev, devs)
    return bytes(out)[:20 * got]


PAGEABLE_FEEDS = {"register": 0, "stage": 1}


def set_pageable_feed(feed):
    """How bt_sha1_chunks_host feeds pageable input >= 64 MiB: "register" (page-lock
    batch by batch, DMA in place; the default) or "stage" (copy into the staging
    lanes).  Returns the previous setting's name."""
    prev = _check(lib.bt_sha1_set_pageable_feed(PAGEABLE_FEEDS[feed]), "bt_sha1_set_pageable_feed")
    return {v: k for k, v in PAGEABLE_FEEDS.items()}[prev]


def pipeline_stats():
    """Phase times and NUMA placement of this thread's last host pipeline run
    (bt_sha1_get_pipeline_stats) as a dict; per-node tallies are trimmed to
    the machine's node count."""
    s = PipelineStats()
    _check(lib.bt_sha1_get_pipeline_stats(ctypes.byref(s)), "bt_sha1_get_pipeline_stats")
    nodes = max(1, min(STATS_NODES, s.numa_nodes))
    d = {k: getattr(s, k) for k, _ in PipelineStats._fields_}
    for k in ("lane_pages", "src_pages", "copy_pieces"):
        d[k] = list(d[k])[:nodes]
    for k in ("total_s", "alloc_s", "fill_s", "wait_s", "register_s", "unregister_s"):
        d[k] = round(d[k], 4)
    d["feed"] = {0: "direct", 1: "staged", 2: "registered"}.get(s.staged, "?")
    d["staged"], d["numa_policy"] = s.staged == 1, {1: "lanes", 2: "gpu"}.get(s.numa_policy, "none")
    return d


def shahash(data):
    """chunk.h:28 through the GPU (aborts the process on a GPU error, like the C call)."""
    buf, n = _host_buf(data)
    out = (ctypes.c_uint8 * 20)()
    lib.shahash(buf, n, out)
    return bytes(out)


class Sha1:
    """SHA1Init/SHA1Update/SHA1Final (sha.h:58-60) on a caller-owned context."""

    def __init__(self):
        self.ctx = SHA1Context()
        lib.SHA1Init(ctypes.byref(self.ctx))

    def update(self, data):
        buf, n = _host_buf(data)
        lib.SHA1Update(ctypes.byref(self.ctx), buf, n)
        return self

    def final(self):
        out = (ctypes.c_uint8 * 20)()
        lib.SHA1Final(ctypes.byref(self.ctx), out)
        return bytes(out)


def binary2hex(b):
    out = ctypes.create_string_buffer(2 * len(b) + 1)
    lib.binary2hex((ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(bytes(b) or b"\0"), len(b), out)
    return out.value.decode()


def hex2binary(h):
    hb = h.encode() if isinstance(h, str) else bytes(h)
    out = (ctypes.c_uint8 * max(len(hb) // 2, 1))()
    lib.hex2binary(ctypes.create_string_buffer(hb, len(hb) + 1), len(hb), out)
    return bytes(out)[:len(hb) // 2]


def make_chunks_file(path, chunk_len=CHUNK):
    """bt_sha1_chunks_file over an open FILE* (libc fopen through ctypes)."""
    libc = ctypes.CDLL(None)
    libc.fopen.restype = _vp
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [_vp]
    size = os.path.getsize(path)
    nch = (size + chunk_len - 1) // chunk_len
    out = (ctypes.c_uint8 * max(20 * nch, 1))()
    fp = libc.fopen(path.encode(), b"rb")
    if not fp:
        raise OSError(f"cannot open {path}")
    try:
        got = _check(lib.bt_sha1_chunks_file(fp, chunk_len, out, nch), "bt_sha1_chunks_file")
    finally:
        libc.fclose(fp)
    raw = bytes(out)
    return [raw[20 * i:20 * i + 20] for i in range(got)]


class Verifier:
    """Batched asynchronous verify (bt_sha1_verifier_*)."""

    def __init__(self, device=0, chunk_len=CHUNK, batch=64, nstreams=2):
        self.h = lib.bt_sha1_verifier_create(device, chunk_len, batch, nstreams)
        if not self.h:
            raise BtSha1Error(f"bt_sha1_verifier_create: {last_error()}")
        self.chunk_len = chunk_len

    def submit(self, chunk, expected, tag):
        buf, n = _host_buf(chunk)
        e = (ctypes.c_uint8 * 20).from_buffer_copy(bytes(expected))
        _check(lib.bt_sha1_verifier_submit(self.h, buf, n, e, tag), "bt_sha1_verifier_submit")

    def slot(self):
        """Hand out a pinned slot (integer address) to assemble a chunk in."""
        p = lib.bt_sha1_verifier_slot(self.h)
        if not p:
            raise BtSha1Error(f"bt_sha1_verifier_slot: {last_error()}")
        return p

    def commit(self, slot, expected, tag, length=None):
        e = (ctypes.c_uint8 * 20).from_buffer_copy(bytes(expected))
        _check(lib.bt_sha1_verifier_commit(self.h, slot, length or self.chunk_len, e, tag),
               "bt_sha1_verifier_commit")

    def release(self, slot):
        _check(lib.bt_sha1_verifier_release(self.h, slot), "bt_sha1_verifier_release")

    def flush(self):
        _check(lib.bt_sha1_verifier_flush(self.h), "bt_sha1_verifier_flush")

    def slot_fill(self, chunk, expected, tag):
        """Zero-copy form: write into a pinned slot, then commit it."""
        p = self.slot()
        ctypes.memmove(p, bytes(chunk), len(chunk))
        self.commit(p, expected, tag, len(chunk))

    def _collect(self, fn, max_n=4096):
        out = (Verdict * max_n)()
        got = _check(fn(self.h, out, max_n), "verifier")
        return [(out[i].tag, bool(out[i].ok), bytes(out[i].digest)) for i in range(got)]

    def poll(self):
        return self._collect(lib.bt_sha1_verifier_poll)

    def drain(self):
        res = []
        while True:
            r = self._collect(lib.bt_sha1_verifier_drain)
            if not r:
                return res
            res += r

    def pending(self):
        return lib.bt_sha1_verifier_pending(self.h)

    def close(self):
        if self.h:
            lib.bt_sha1_verifier_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
