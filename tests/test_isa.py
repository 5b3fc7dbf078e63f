"""CPU: the hot kernel's compiled gfx950 code has the instruction mix DESIGN.md §4
claims (597 VALU per 64-byte block, no scratch, registers within 2 waves/SIMD),
and the schedule identity the shared-pair form rests on holds."""
import importlib.util
import os
import random

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _isa_mix():
    spec = importlib.util.spec_from_file_location("isa_mix", os.path.join(REPO, "tools", "isa_mix.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc absent")
    mod = _isa_mix()
    out = str(tmp_path_factory.mktemp("isa") / "k.s")
    mod.compile_asm(out)
    return mod, open(out).read()


@pytest.mark.parametrize("nbuf,lines", [(3, 1), (2, 1), (4, 1), (2, 2)])
def test_hot_loop_mix(asm, nbuf, lines):
    mod, text = asm
    m = mod.loop_mix(text, nbuf, lines)
    assert m["valu_per_block"] == 597, m
    assert m["half_rate_per_block"] == 400 and m["full_rate_per_block"] == 197, m
    assert m["mix_per_block"]["v_xor_b32_e32"] == 48 and m["mix_per_block"]["v_alignbit_b32"] == 224, m
    assert m["scratch_bytes"] == 0 and m["vgprs"] <= 256, m


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def test_schedule_squared_twice_identity():
    """W[t] = ROTL4(W[t-12]^W[t-32]^W[t-56]^W[t-64]) for t >= 64 and
    ROTL2(W[t-6]^W[t-16]^W[t-28]^W[t-32]) for t >= 32, given the sha.c:196-200
    recurrence -- what sched_pair (sha1_device.h) relies on."""
    rng = random.Random(7)
    for _ in range(200):
        w = [rng.getrandbits(32) for _ in range(16)]
        for t in range(16, 80):
            w.append(_rotl(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1))
        for t in range(32, 80):
            assert w[t] == _rotl(w[t - 6] ^ w[t - 16] ^ w[t - 28] ^ w[t - 32], 2)
        for t in range(64, 80):
            assert w[t] == _rotl(w[t - 12] ^ w[t - 32] ^ w[t - 56] ^ w[t - 64], 4)


def _first_wait_after_each_load_group(text, sym):
    """For every run of 16-byte global loads in kernel `sym`, the vmcnt of the
    first s_waitcnt that follows it."""
    import re
    body = text[text.index(sym + ":"):]
    body = body[:body.index(".Lfunc_end")]
    out, in_group = [], False
    for line in body.splitlines():
        line = line.strip()
        if line.startswith("global_load_dwordx4"):
            in_group = True
            continue
        m = re.match(r"s_waitcnt vmcnt\((\d+)\)", line)
        if m and in_group:
            out.append(int(m.group(1)))
            in_group = False
    return out


@pytest.mark.parametrize("sym", ["_ZN6btsha113k_sha1_raggedEPKhPKmPKjmjmPh", "_ZN6btsha115k_sha1_midstateEPjPKhm"])
def test_ragged_ring_keeps_loads_in_flight(asm, sym):
    """The generic kernels' prefetch ring (absorb_ring) must not wait for the
    block it just asked for: the first wait after each group of four 16-byte
    loads leaves that whole group outstanding (vmcnt >= 4).  A guarded
    (branched) prefetch made hipcc wait vmcnt(3..0) right after issuing it --
    one memory round trip per block."""
    _, text = asm
    waits = _first_wait_after_each_load_group(text, sym)
    assert waits, "no 16-byte load groups found"
    assert min(waits) >= 4, waits
