"""oracle/py_oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes access to the CPU checkers:
  * liboracle_sha1.so   our restatement of the reference (oracle/sha1_oracle.c)
  * _ref/libref_sha1.so the reference's own chunk.c + sha.c, compiled from
                        /root/reference by oracle/Makefile (present only where it
                        was built; travels to the GPU box as a prebuilt file)
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (libbtsha1.so) never does.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle_sha1.so")
REF_SO = os.path.join(HERE, "_ref", "libref_sha1.so")
REF_SO_O0 = os.path.join(HERE, "_ref", "libref_sha1_O0.so")

_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64

_lib = ctypes.CDLL(ORACLE_SO)
_lib.or_shahash.argtypes = [_vp, ctypes.c_int, _vp]
_lib.or_fill_synthetic.argtypes = [_vp, _u64, _u64, _u64]
_lib.or_hash_chunks.argtypes = [_vp, _u64, _u64, ctypes.c_uint32, ctypes.c_uint32, _vp, ctypes.c_int]
_lib.or_hash_chunks.restype = ctypes.c_int
_lib.or_sha1_init.argtypes = [_vp]
_lib.or_sha1_update.argtypes = [_vp, _vp, ctypes.c_uint32]
_lib.or_sha1_final.argtypes = [_vp, _vp]
_lib.or_sha1_blocks.argtypes = [_vp, _vp, _u64]
_lib.or_binary2hex.argtypes = [_vp, ctypes.c_int, ctypes.c_char_p]
_lib.or_hex2binary.argtypes = [ctypes.c_char_p, ctypes.c_int, _vp]
_lib.or_synth_digests.argtypes = [_u64, _u64, ctypes.c_uint32, _u64, _vp, ctypes.c_int]
_lib.or_synth_digests.restype = ctypes.c_int

SEED_SYNTH = 0x0B175EED
SEED_EDGE = 0x5EED0001
SEED_TAIL = 0x7A11
SEED_RAGGED = 0xABCD
CHUNK = 512 * 1024


def ragged_len(k):
    """Length of message k of the committed ragged golden batch (tests/golden/make_golden.py)."""
    return (k * 7919) % 2113 + (k % 5) * 64


def _buf(data):
    return (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(bytes(data) or b"\0")


def sha1(data) -> bytes:
    out = (ctypes.c_uint8 * 20)()
    _lib.or_shahash(_buf(data), len(data), out)
    return bytes(out)


class Sha1Stream:
    def __init__(self):
        self.ctx = ctypes.create_string_buffer(128)
        _lib.or_sha1_init(self.ctx)

    def update(self, data):
        _lib.or_sha1_update(self.ctx, _buf(data), len(data))
        return self

    def final(self):
        out = (ctypes.c_uint8 * 20)()
        _lib.or_sha1_final(self.ctx, out)
        return bytes(out)


def fill_synthetic(nbytes, first_word, seed) -> bytearray:
    buf = bytearray(max(nbytes, 1))
    arr = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    _lib.or_fill_synthetic(arr, nbytes, first_word, seed)
    return buf[:nbytes] if nbytes else bytearray()


def hash_chunks(data, chunk_len, pitch=None, nthreads=1, lib=None):
    """Digests of equal chunks (short last one) in a host buffer, pthread-split."""
    n_bytes = len(data)
    pitch = pitch or chunk_len
    n = (n_bytes + pitch - 1) // pitch if n_bytes else 0
    last = n_bytes - (n - 1) * pitch if n else 0
    last = min(last, chunk_len)
    out = (ctypes.c_uint8 * max(20 * n, 1))()
    if isinstance(data, bytearray):
        src = (ctypes.c_uint8 * len(data)).from_buffer(data)
    else:
        src = _buf(data)
    if _lib.or_hash_chunks(src, n, pitch, chunk_len, last, out, nthreads):
        raise RuntimeError("or_hash_chunks failed (out of memory, or a worker thread could not be created)")
    raw = bytes(out)
    return [raw[20 * i:20 * i + 20] for i in range(n)]


def usable_cpus():
    """CPUs this process may actually use: the affinity mask capped by the
    cgroup CPU quota (a GPU box shows 256 CPUs but pays for 16)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = max(1, min(n, -(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def synth_digests(first_chunk, n, chunk_len=CHUNK, seed=SEED_SYNTH, nthreads=None) -> bytes:
    """20-byte digests of synthetic chunks first_chunk .. first_chunk+n-1 (chunk g
    = stream words [g*chunk_len/8, ..), as bench.py and the tests lay them out),
    each regenerated and hashed in C across threads: every digest of a 64 GiB
    batch in seconds, with no image in memory."""
    out = (ctypes.c_uint8 * max(20 * n, 1))()
    if _lib.or_synth_digests(first_chunk, n, chunk_len, seed, out, nthreads or usable_cpus()):
        raise ValueError("or_synth_digests failed (chunk_len must be a multiple of 8; or out of memory, "
                         "or a worker thread could not be created)")
    return bytes(out)[:20 * n]


def binary2hex(b) -> str:
    out = ctypes.create_string_buffer(2 * len(b) + 1)
    _lib.or_binary2hex(_buf(b), len(b), out)
    return out.value.decode()


def hex2binary(h) -> bytes:
    hb = h.encode() if isinstance(h, str) else bytes(h)
    out = (ctypes.c_uint8 * max(len(hb) // 2, 1))()
    _lib.or_hex2binary(ctypes.create_string_buffer(hb, len(hb) + 1), len(hb), out)
    return bytes(out)[:len(hb) // 2]


def compress_blocks(state, blocks: bytes):
    st = (ctypes.c_uint32 * 5)(*state)
    _lib.or_sha1_blocks(st, _buf(blocks), len(blocks) // 64)
    return list(st)


ORACLE_SO_O0 = os.path.join(HERE, "liboracle_sha1_O0.so")


def load_port(opt="O2"):
    """Our restatement as a shahash-compatible library: or_shahash(buf, len, out)
    (-O2 build, or the -O0 one matching the reference Makefile's flags)."""
    if opt == "O2":
        return _lib
    if not os.path.exists(ORACLE_SO_O0):
        return None
    lib = ctypes.CDLL(ORACLE_SO_O0)
    lib.or_shahash.argtypes = [_vp, ctypes.c_int, _vp]
    lib.or_shahash.restype = None
    return lib


def load_reference(opt="O2"):
    """The reference's shahash from oracle/_ref (None when not built here)."""
    path = REF_SO if opt == "O2" else REF_SO_O0
    if not os.path.exists(path):
        return None
    ref = ctypes.CDLL(path)
    ref.shahash.argtypes = [_vp, ctypes.c_int, _vp]
    ref.shahash.restype = None
    return ref
