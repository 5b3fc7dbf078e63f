"""CPU: the C-ABI library builds, loads, exports every declared entry point,
and fails loudly (not silently, not on the CPU) when no GPU is present."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

from conftest import REPO, PKG, load_btsha1

LIB = os.path.join(PKG, "libbtsha1.so")
HEADERS = [os.path.join(REPO, "include", h) for h in ("bt_sha1.h", "sha.h", "chunk.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", text, flags=re.M):
            if not m.group(0).lstrip().startswith(("#", "typedef")):
                names.add(m.group(1))
    return names


def test_headers_declare_reference_surface():
    names = declared_functions()
    # sha.h:58-60 and chunk.h:25-34 of the reference
    for ref in ["SHA1Init", "SHA1Update", "SHA1Final", "make_chunks", "shahash", "binary2hex", "hex2binary"]:
        assert ref in names
    assert len(names) > 25


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "run make first"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = declared_functions() - exported
    assert not missing, missing


def test_library_is_gfx950_code_object():
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"k_sha1_fixed" in blob


def test_loads_and_reports_no_device_loudly():
    bt = load_btsha1()
    if bt.device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    with pytest.raises(bt.BtSha1Error, match="device"):
        bt.chunks_host(b"x" * 100, 64)
    assert "gfx950" in bt.build_info()


def test_dropin_void_calls_abort_without_gpu(tmp_path):
    """shahash cannot return an error (chunk.h:28): it must abort, never hash on the CPU."""
    code = ("import ctypes,sys; l=ctypes.CDLL(sys.argv[1]); o=(ctypes.c_uint8*20)(); "
            "l.shahash(b'abc', 3, o); print('returned', bytes(o).hex())")
    r = subprocess.run([sys.executable, "-c", code, LIB], capture_output=True, text=True)
    if "returned" in r.stdout and r.returncode == 0:
        pytest.skip("GPU visible")
    assert r.returncode != 0
    assert "libbtsha1: shahash" in r.stderr


def test_worker_list_is_bounded():
    """bt_sha1_chunks_host_devices: each worker is a host thread with its own
    staging lanes, so the list is capped (checked before any device call)."""
    bt = load_btsha1()
    with pytest.raises(bt.BtSha1Error, match="at most 64"):
        bt.chunks_host(b"x" * 100, 64, devs=[0] * 65)
    with pytest.raises(bt.BtSha1Error, match="empty device list"):
        bt.chunks_host(b"x" * 100, 64, devs=[])


def test_barrier_tallies_only_in_the_debug_build():
    """bt_sha1_debug_barrier_stats reports -1 in the production library (no HIP
    call is made); the barrier-accounting build (make dbgbar, exercised by
    tests/test_gpu_barriers.py) carries the device tallies."""
    bt = load_btsha1()
    with pytest.raises(bt.BtSha1Error, match="dbgbar"):
        bt.debug_barrier_stats()
    dbg = os.path.join(REPO, "build_variants", "dbgbar", "libbtsha1.so")
    assert os.path.exists(dbg), "run make dbgbar first"
    assert b"g_bar_stats" in open(dbg, "rb").read()
    assert b"g_bar_stats" not in open(LIB, "rb").read()


def test_dropin_residue_hook_needs_no_device():
    """bt_sha1_debug_dropin_residue (the wipe-contract probe, chunk.c:48):
    nothing staged before any drop-in call -> 0, a negative device -> -1,
    with no HIP call made (the GPU tests check it reads 0 after real calls)."""
    bt = load_btsha1()
    assert bt.debug_dropin_residue(0) == 0
    with pytest.raises(bt.BtSha1Error, match="out of range"):
        bt.debug_dropin_residue(-1)


def test_pipeline_stats_layout_and_no_run_error(tmp_path):
    """bt_sha1_pipeline_stats: the ctypes mirror btsha1.PipelineStats has the
    C struct's size and field offsets (compiled here against
    include/bt_sha1.h), and a thread that has run no host pipeline gets -1
    with a message, not stale numbers."""
    import threading
    bt = load_btsha1()
    fields = [f for f, _ in bt.PipelineStats._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "bt_sha1.h"\nint main(void) {\n'
                   '  printf("size %zu\\n", sizeof(bt_sha1_pipeline_stats));\n'
                   + "".join(f'  printf("{f} %zu\\n", offsetof(bt_sha1_pipeline_stats, {f}));\n' for f in fields)
                   + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(src)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True)
               .stdout.splitlines())
    assert int(got["size"]) == ctypes.sizeof(bt.PipelineStats)
    for f in fields:
        assert int(got[f]) == getattr(bt.PipelineStats, f).offset, f
    err = []

    def fresh_thread():
        try:
            bt.pipeline_stats()
        except bt.BtSha1Error as e:
            err.append(str(e))
    t = threading.Thread(target=fresh_thread)
    t.start()
    t.join()
    assert err and "no host pipeline has run on this thread" in err[0]


EXP_LIB = os.path.join(REPO, "build_variants", "experiments", "libbtsha1.so")


def _kernel_symbols(lib):
    """Mangled kernel names in a library's gfx950 code object."""
    blob = open(lib, "rb").read()
    return set(m.decode() for m in re.findall(rb"_ZN6btsha1\d+k_sha1_\w+?(?=\x00|\.kd)", blob))


def test_product_library_carries_only_the_default_hot_kernel():
    """One compression, one hot path in the product (sha.c:176-451): the
    rejected ring / nt / LDS-staged variants live only in the experiments
    library, and the product's bt_sha1_set_variant refuses them (no device
    call is made, so this runs without a GPU)."""
    bt = load_btsha1()
    for v in ((4, 1, 0), (2, 1, 0), (2, 2, 0), (3, 1, 1), (10, 1, 0), (10, 1, 1)):
        with pytest.raises(bt.BtSha1Error, match="experiments"):
            bt.set_variant(*v)
    bt.set_variant(3, 1, 0)  # the default stays selectable
    prod = _kernel_symbols(LIB)
    fixed = {s for s in prod if "k_sha1_fixed" in s}
    assert fixed and all("ILi3ELi1ELi0E" in s for s in fixed), fixed
    assert not any("k_sha1_lds" in s for s in prod), prod
    assert os.path.exists(EXP_LIB), "run make experiments first"
    exp = _kernel_symbols(EXP_LIB)
    assert any("k_sha1_lds" in s for s in exp) and any("ILi4ELi1ELi0E" in s for s in exp)
    assert os.path.getsize(LIB) < 0.5 * os.path.getsize(EXP_LIB)


def test_diagnostic_builds_carry_their_own_source_id():
    """bench.py reuses PMC traffic only for the source id it was measured on:
    every diagnostic / experiment build reports a suffixed id."""
    prod = subprocess.run([sys.executable, "-c", "import ctypes,sys; l=ctypes.CDLL(sys.argv[1]); "
                           "l.bt_sha1_source_id.restype=ctypes.c_char_p; print(l.bt_sha1_source_id().decode())", LIB],
                          capture_output=True, text=True, check=True).stdout.strip()
    for name, suffix in (("experiments", "-exp"), ("dbgbar", "-dbgbar")):
        lib = os.path.join(REPO, "build_variants", name, "libbtsha1.so")
        out = subprocess.run([sys.executable, "-c", "import ctypes,sys; l=ctypes.CDLL(sys.argv[1]); "
                              "l.bt_sha1_source_id.restype=ctypes.c_char_p; print(l.bt_sha1_source_id().decode())",
                              lib], capture_output=True, text=True, check=True).stdout.strip()
        assert out == prod + suffix, (name, out, prod)


def test_sha1context_layout_matches_reference():
    bt = load_btsha1()
    # sha.h:39-50 of the reference: u64 + 5*u32 + u32 + 64-byte union = 96 bytes
    assert ctypes.sizeof(bt.SHA1Context) == 96
    assert bt.SHA1Context.buffer.offset == 32


def test_hex_codec_is_host_formatting():
    bt = load_btsha1()
    b = bytes(range(20))
    assert bt.binary2hex(b) == b.hex()
    assert bt.hex2binary(b.hex()) == b
    assert bt.hex2binary("0g") == bytes([16])  # bug-compatible with chunk.c:66-71


def test_reference_callers_compile_and_link_against_dropin(tmp_path):
    """make_chunks.c and chunk-using code of the reference build unchanged
    against include/ + libbtsha1.so (the drop-in claim)."""
    src = "/root/reference/make_chunks.c"
    if not os.path.exists(src):
        pytest.skip("reference sources absent (GPU box)")
    exe = tmp_path / "make-chunks-dropin"
    subprocess.run(["gcc", "-Wall", "-I", os.path.join(REPO, "include"), "-o", str(exe), src,
                    f"-L{PKG}", "-lbtsha1", "-lm", f"-Wl,-rpath,{PKG}"], check=True, capture_output=True)
    assert exe.exists()


def test_integration_peer_example_compiles(tmp_path):
    """The batched-verify snippet of INTEGRATION.md §3 compiles and links against
    include/ + libbtsha1.so as written, over the reference's own Chunk /
    Request layout (guards the documented calls against drift); its per-chunk
    table is sized from the request, never a fixed array indexed by chunk id."""
    import re
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = text[text.index("## 3."):]
    body = re.search(r"```c\n(.*?)```", sec, re.S).group(1)
    body = "\n".join(l for l in body.splitlines() if not l.startswith("#include"))
    src = tmp_path / "peer_example.c"
    src.write_text(
        "#include <stdint.h>\n#include <stdlib.h>\n#include \"bt_sha1.h\"\n#include \"chunk.h\"\n"
        "enum { NOT_STARTED, RECEIVING, VERIFYING, OWNED };\n"
        "struct Chunk { int id; uint8_t hash[20]; int state; char *data; int received_seq_number;\n"
        "               int received_byte_number; };\n"          # common.h:45-52
        "struct Request { char *filename; int chunk_number; struct Chunk *chunks; };\n"  # common.h:54-58
        "void peer_example(struct Chunk *chunk, int chunk_id, struct Request *current_request) {\n"
        + body + "\n}\nint main(void) { return 0; }\n")
    exe = tmp_path / "peer_example"
    assert "calloc((size_t)current_request->chunk_number" in body and not re.search(r"static[^;]*\[\d+\];", body)
    r = subprocess.run(["gcc", "-Wall", "-Wno-unused-variable", "-Werror", "-I", os.path.join(REPO, "include"),
                        "-o", str(exe), str(src), f"-L{PKG}", "-lbtsha1", f"-Wl,-rpath,{PKG}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_make_install_tree_links_a_reference_style_caller(tmp_path):
    """`make install PREFIX=...` gives the layout a reference build links
    against: the library, the drop-in headers, the CLIs
    and a pkg-config file whose flags build a chunk.h / sha.h caller."""
    prefix = tmp_path / "inst"
    r = subprocess.run(["make", "-C", REPO, "install", f"PREFIX={prefix}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    for f in ("lib/libbtsha1.so", "include/sha.h", "include/chunk.h", "include/bt_sha1.h",
              "bin/make-chunks", "bin/verify-stream", "lib/pkgconfig/btsha1.pc"):
        assert (prefix / f).exists(), f
    pc = dict(l.split("=", 1) for l in (prefix / "lib/pkgconfig/btsha1.pc").read_text().splitlines()
              if "=" in l and ":" not in l.split("=", 1)[0])
    assert pc["prefix"] == str(prefix)
    src = tmp_path / "caller.c"
    src.write_text('#include <stdio.h>\n#include "chunk.h"\n#include "sha.h"\n'
                   "int main(int c, char **v) { uint8_t *h[1]; uint8_t d[20]; SHA1Context s; SHA1Init(&s);\n"
                   "  if (c > 5) { FILE *f = fopen(v[1], \"rb\"); h[0] = d; return make_chunks(f, h); }\n"
                   "  return 0; }\n")
    exe = tmp_path / "caller"
    r = subprocess.run(["gcc", "-Wall", "-Werror", f"-I{prefix}/include", "-o", str(exe), str(src),
                        f"-L{prefix}/lib", "-lbtsha1", f"-Wl,-rpath,{prefix}/lib"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    ldd = subprocess.run(["ldd", str(exe)], capture_output=True, text=True).stdout
    assert f"{prefix}/lib/libbtsha1.so" in ldd
    ldd = subprocess.run(["ldd", str(prefix / "bin" / "make-chunks")], capture_output=True, text=True).stdout
    assert f"{prefix}/lib/libbtsha1.so" in ldd


@pytest.mark.parametrize("args,msg", [
    (["-r", "2", "-w", "2"], "no timed round"),
    (["-r", "0"], "usage"),
    (["-g", "65"], "usage"),
    (["-w", "-1"], "usage"),
    (["-q"], "usage"),
])
def test_verify_stream_rejects_bad_options_before_any_gpu_call(tmp_path, args, msg):
    """bin/verify-stream's option checks (-w warm-up rounds must leave a timed
    round, -r >= 1, 1 <= -g <= 64) fail with status 255 and a message before
    the data files are opened or a device is touched -- so they hold on a
    machine without a GPU."""
    exe = os.path.join(PKG, "bin", "verify-stream")
    assert os.path.exists(exe), "run make tools first"
    r = subprocess.run([exe, *args, str(tmp_path / "missing.img"), str(tmp_path / "missing.chunks")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 255 and msg in r.stderr, (r.returncode, r.stderr)


def test_chunk_len_checked_before_any_chunk_arithmetic():
    """bt_sha1_chunks_host with chunk_len 0 or >= 4 GiB (the kernels' 32-bit
    lengths) is -1 with a message, before any device call or division by the
    chunk length."""
    bt = load_btsha1()
    buf = (ctypes.c_uint8 * 4096)()
    out = (ctypes.c_uint8 * 20)()
    for cl in (0, 1 << 32):
        assert bt.lib.bt_sha1_chunks_host(buf, 4096, cl, out) == -1, cl
        assert "chunk_len must be in [1, 4 GiB)" in bt.last_error(), cl


def test_pageable_feed_switch_needs_no_device():
    """bt_sha1_set_pageable_feed: REGISTER (0, the default) / STAGE (1) swap
    and report the previous setting; anything else is -1 with a message; no
    device call is made."""
    bt = load_btsha1()
    prev = bt.set_pageable_feed("stage")
    assert prev in ("register", "stage")
    assert bt.set_pageable_feed("register") == "stage"
    assert bt.lib.bt_sha1_set_pageable_feed(7) == -1 and "BT_SHA1_PAGEABLE_STAGE" in bt.last_error()
    bt.set_pageable_feed(prev)
