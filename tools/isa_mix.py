#!/usr/bin/env python3
"""isa_mix.py -- VALU instruction mix per 64-byte block of the hot kernel, read
from the gfx950 ISA that hipcc emits for sha1_kernels.hip.

The hot loop of k_sha1_fixed<NBUF, L, 0, false> compresses NBUF*2L blocks per
iteration (fully unrolled), so the per-block mix is the loop body's count
divided by that.  Also reports the kernel's VGPR count and scratch size.
Usage: python3 tools/isa_mix.py [NBUF L]   (default: 3 1, the library default;
other shapes are read from the experiments build)
Prints one JSON object.  DESIGN.md §4 quotes these numbers; tests/test_isa.py
checks them.
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(HERE, "bittorrent-with-congestion-control_amd", "csrc")

HALF_RATE = {"v_alignbit_b32", "v_add3_u32", "v_perm_b32"}  # tools/ubench/valu_rate.hip


def compile_asm(out, experiments=False):
    """Device ISA of sha1_kernels.hip as the product library builds it, or with
    the rejected hot-kernel variants too (the experiments library)."""
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-I" + os.path.join(HERE, "include"), "-I" + CSRC, "--cuda-device-only", "-S",
                    *(["-DBT_SHA1_EXPERIMENTS"] if experiments else []),
                    "-o", out, os.path.join(CSRC, "sha1_kernels.hip")],
                   check=True, capture_output=True)


def fixed_symbol(nbuf, lines, stamp=False):
    """Mangled name of k_sha1_fixed<nbuf, lines, 0, false, stamp>."""
    return f"_ZN6btsha112k_sha1_fixedILi{nbuf}ELi{lines}ELi0ELb0ELb{int(stamp)}EEEvPKhmjjPhS2_S3_jPm"


def loop_mix(asm_text, nbuf, lines, stamp=False):
    sym = fixed_symbol(nbuf, lines, stamp)
    start = asm_text.index(sym + ":")
    body = asm_text[start:]
    end_fn = body.index(".Lfunc_end")
    body = body[:end_fn]
    m = re.search(r"^(\.LBB\d+_\d+):[^\n]*Inner Loop Header", body, re.M)
    label = m.group(1)
    loop = body[m.end():body.index(f"s_cbranch_scc1 {label}", m.end())]
    ops = collections.Counter()
    for line in loop.splitlines():
        line = line.strip()
        if line.startswith("v_"):
            ops[line.split()[0]] += 1
    blocks = nbuf * 2 * lines
    meta = asm_text[start:]
    vgprs = int(re.search(r"; NumVgprs: (\d+)", meta).group(1))
    scratch = int(re.search(r"; ScratchSize: (\d+)", meta).group(1))
    per_block = {k: v / blocks for k, v in sorted(ops.items())}
    total = sum(per_block.values())
    half = sum(v for k, v in per_block.items() if k in HALF_RATE)
    return {"kernel": f"k_sha1_fixed<{nbuf},{lines},0,false,{str(stamp).lower()}>", "blocks_per_iteration": blocks,
            "valu_per_block": total, "half_rate_per_block": half, "full_rate_per_block": total - half,
            "mix_per_block": per_block, "vgprs": vgprs, "scratch_bytes": scratch}


def main():
    nbuf, lines = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (3, 1)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        compile_asm(out, experiments=(nbuf, lines) != (3, 1))
        print(json.dumps(loop_mix(open(out).read(), nbuf, lines)))


if __name__ == "__main__":
    main()
