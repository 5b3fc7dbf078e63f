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


@pytest.fixture(scope="module")
def asm_exp(tmp_path_factory):
    """The experiments library's kernels (rejected ring shapes, nt, LDS)."""
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc absent")
    mod = _isa_mix()
    out = str(tmp_path_factory.mktemp("isa_exp") / "k.s")
    mod.compile_asm(out, experiments=True)
    return mod, open(out).read()


def test_hot_loop_mix(asm):
    mod, text = asm
    _check_mix(mod.loop_mix(text, 3, 1))


@pytest.mark.parametrize("nbuf,lines", [(3, 1), (2, 1), (4, 1), (2, 2)])
def test_hot_loop_mix_experiment_variants(asm_exp, nbuf, lines):
    """Every ring shape of the experiments build compresses with the same
    597-instruction block (DESIGN.md §5 compares them at equal work)."""
    mod, text = asm_exp
    _check_mix(mod.loop_mix(text, nbuf, lines))


def test_product_hot_kernel_is_the_experiments_default(asm, asm_exp):
    """The product's k_sha1_fixed<3,1,...> is instruction for instruction the
    experiments build's, so measurements of either apply to both."""
    import re
    mod, text = asm
    _, etext = asm_exp

    def body(t, sym):
        b = t[t.index(sym + ":"):]
        b = b[:b.index(".Lfunc_end")]
        return [re.sub(r"BB\d+_", "BB_", l.split(";")[0].strip()) for l in b.splitlines() if l.split(";")[0].strip()]
    sym = mod.fixed_symbol(3, 1)
    assert body(text, sym) == body(etext, sym)
    assert "k_sha1_lds" not in text and mod.fixed_symbol(4, 1) not in text


def _check_mix(m):
    assert m["valu_per_block"] == 597, m
    assert m["half_rate_per_block"] == 400 and m["full_rate_per_block"] == 197, m
    assert m["mix_per_block"]["v_xor_b32_e32"] == 48 and m["mix_per_block"]["v_alignbit_b32"] == 224, m
    assert m["scratch_bytes"] == 0 and m["vgprs"] <= 256, m


def test_clock_probe_build_runs_the_same_loop(asm):
    """bench.py's clock probe (bt_sha1_clock_probe) times the STAMP build of the
    hot kernel: its main loop must be the production loop, instruction for
    instruction, so the clock it reads is the clock the benchmark runs at."""
    mod, text = asm
    prod = mod.loop_mix(text, 3, 1)
    stamped = mod.loop_mix(text, 3, 1, stamp=True)
    assert stamped["mix_per_block"] == prod["mix_per_block"], (stamped, prod)
    body = text[text.index(mod.fixed_symbol(3, 1, True) + ":"):]
    body = body[:body.index(".Lfunc_end")]
    assert body.count("s_memtime") == 2 and body.count("s_memrealtime") == 2
    prod_body = text[text.index(mod.fixed_symbol(3, 1) + ":"):]
    assert "s_memtime" not in prod_body[:prod_body.index(".Lfunc_end")]


def test_no_scalar_stores_anywhere(asm):
    """No kernel writes through the scalar data cache (gpurun refuses such code)."""
    import re
    _, text = asm
    # scalar stores (plain / buffer / scratch), scalar atomics, scalar-cache writeback or discard
    pattern = r"^\s*s_(?:(?:buffer_|scratch_)?store|atomic|dcache_(?:wb|discard))"
    assert not re.search(pattern, text, re.M)


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


def _first_wait_after_each_load_group(text, sym, load="global_load_dwordx4"):
    """For every run of 16-byte loads in kernel `sym`, the vmcnt of the
    first s_waitcnt that follows it."""
    import re
    body = text[text.index(sym + ":"):]
    body = body[:body.index(".Lfunc_end")]
    out, in_group = [], False
    for line in body.splitlines():
        line = line.strip()
        if line.startswith(load):
            in_group = True
            continue
        m = re.match(r"s_waitcnt vmcnt\((\d+)\)", line)
        if m and in_group:
            out.append(int(m.group(1)))
            in_group = False
    return out


@pytest.mark.parametrize("sym", ["_ZN6btsha113k_sha1_raggedEPKhPKmPKjmjmPh"])
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


def _sym(text, prefix):
    """The one kernel symbol that starts with `prefix` (mangled template args)."""
    import re
    found = sorted(set(re.findall(r"^(" + re.escape(prefix) + r"\w*):", text, re.M)))
    assert len(found) == 1, found
    return found[0]


LAT_SYM = "_ZN6btsha110k_sha1_latILb0ELi2ELi0EE"  # k_sha1_lat<false, 2 slots, whole chunks>
# its column forms (first / middle / last column of the host pipelines'
# column-split tail): the same round wave
LAT_COLUMN_SYMS = ["_ZN6btsha110k_sha1_latILb0ELi2ELi%dEE" % m for m in (1, 2, 3)]


def _loops(text, sym):
    """(header label, body text) of every innermost loop of kernel `sym`."""
    import re
    body = text[text.index(sym + ":"):]
    body = body[:body.index(".Lfunc_end")]
    out = []
    # the header comment sits on the label's line or, for nested loops, the next one
    for m in re.finditer(r"^(\.LBB\d+_\d+):[^\n]*(?:\n\s*;[^\n]*)?Inner Loop Header", body, re.M):
        label = m.group(1)
        end = re.search(r"s_cbranch_\w+ " + re.escape(label) + r"\b", body[m.end():])
        if end:  # loops entered by fall-through from a latch block are not innermost-simple
            out.append((label, body[m.end():m.end() + end.start()]))
    return out


@pytest.mark.parametrize("prefix", [LAT_SYM] + LAT_COLUMN_SYMS)
def test_latency_kernel_round_wave_structure(asm, prefix):
    """k_sha1_lat: the round wave R's loop is one 64-byte block
    per iteration with 5 VALU per round (+ the 5 state adds) = 405, its 80 W+K
    words read as 20 ds_read_b128 from ONE 80-word LDS slot, and exactly one
    s_barrier (the loader wave S pairs it with one barrier per block).  This
    layout was once lost in a revert and caught only by re-timing.  The
    column forms (chaining state in / out instead of IV / digest) keep it."""
    import collections
    _, text = asm
    r_loops = [b for _, b in _loops(text, _sym(text, prefix)) if "ds_read_b128" in b and "buffer_load" not in b]
    assert len(r_loops) == 1, len(r_loops)
    ops = collections.Counter(l.strip().split()[0] for l in r_loops[0].splitlines()
                              if l.strip() and not l.strip().startswith((".", ";")))
    valu = sum(v for k, v in ops.items() if k.startswith("v_"))
    assert valu == 405, ops
    assert ops["ds_read_b128"] == 20 and ops["s_barrier"] == 1, ops
    assert ops["v_alignbit_b32"] == 160 and ops["v_bitop3_b32"] == 80, ops


@pytest.mark.parametrize("prefix", [LAT_SYM] + LAT_COLUMN_SYMS)
def test_latency_kernel_loader_ring_keeps_loads_in_flight(asm, prefix):
    """S's four-block register ring never waits for the block it just issued:
    the first wait after each group of 16-byte buffer loads leaves >= 4 of them
    outstanding (a vmcnt(0) there would put a memory round trip on every block
    R waits for at the barrier)."""
    _, text = asm
    waits = _first_wait_after_each_load_group(text, _sym(text, prefix), load="buffer_load_dwordx4")
    assert waits, "no buffer load groups found"
    assert min(waits) >= 4, waits


CHAIN_SYM = "_ZN6btsha112k_sha1_chainILb0ELb0EE"  # k_sha1_chain<false, false>


def test_chain_kernel_round_wave_structure(asm):
    """k_sha1_chain's round wave: per block two ds_read_b128
    (lanes 0..15 / 0..3 hold the block's 80 W+K words) and one add per round
    fed by a DPP row shift from the lane that holds the word, so the loop is
    ~405 VALU with no per-round LDS traffic (the broadcast form had 20
    ds_read_b128 and ~8 waits per block)."""
    import collections
    _, text = asm
    loops = [b for _, b in _loops(text, _sym(text, CHAIN_SYM)) if "v_alignbit_b32" in b]
    assert len(loops) == 1, len(loops)
    ops = collections.Counter(l.strip().split()[0] for l in loops[0].splitlines()
                              if l.strip() and not l.strip().startswith((".", ";")))
    valu = sum(v for k, v in ops.items() if k.startswith("v_"))
    assert 405 <= valu <= 410, ops
    assert ops["ds_read_b128"] == 2 and ops["v_add_u32_dpp"] >= 70, ops
    assert ops["v_alignbit_b32"] == 160 and ops["v_bitop3_b32"] == 80, ops



LAT_RAGGED = ["_ZN6btsha117k_sha1_lat_raggedILi2EE", "_ZN6btsha117k_sha1_lat_raggedILi3EE"]


@pytest.mark.parametrize("prefix", LAT_RAGGED)
def test_ragged_latency_loader_ring_keeps_loads_in_flight(asm, prefix):
    """k_sha1_lat_ragged's loader wave reads each lane's own message through a
    four-block register ring (messages of unequal length, so global loads, not
    buffer loads): no wait right after a group of 16-byte loads may drain it
    (vmcnt >= 4); the tail words are hoisted out of the per-block branch."""
    _, text = asm
    waits = _first_wait_after_each_load_group(text, _sym(text, prefix))
    assert waits, "no 16-byte load groups found"
    assert min(waits) >= 4, waits


def test_ragged_latency_round_wave_structure(asm):
    """Its round wave is k_sha1_lat's (405 VALU per block, 20 ds_read_b128
    from one 80-word slot, one s_barrier) plus a handful of selects that latch
    each lane's state at its own last block."""
    import collections
    _, text = asm
    r_loops = [b for _, b in _loops(text, _sym(text, LAT_RAGGED[0])) if "ds_read_b128" in b]
    assert len(r_loops) == 1, len(r_loops)
    ops = collections.Counter(l.strip().split()[0] for l in r_loops[0].splitlines()
                              if l.strip() and not l.strip().startswith((".", ";")))
    valu = sum(v for k, v in ops.items() if k.startswith("v_"))
    assert 405 <= valu <= 415, ops
    assert ops["ds_read_b128"] == 20 and ops["s_barrier"] == 1, ops
