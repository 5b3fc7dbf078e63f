"""CPU: .chunks text formats through libbtsha1's host-side
parsers, pinned on the reference's own fixture files."""
import os

import pytest

from conftest import GOLDEN, load_btsha1, read_pairs

C_DIGESTS = ["6acfce07d222d400ce900d918306c6664501b33f", "af91dbd47aac60e980e0369df68271ca52de11a8",
             "3b9f916bbf59021ab781c9f2456df90a0102079f", "78585121ee33fbb6666bc4bf1a8498c04b2758e8"]


@pytest.fixture(scope="module")
def bt():
    return load_btsha1()


def test_master_file_of_reference(bt):
    # p2-tests/C.chunks: "File: C.tar" / "Chunks:" + 4 lines (util.c:113-164, peer.c:299-305)
    name, entries = bt.parse_master(os.path.join(GOLDEN, "ref_C.chunks"))
    assert name == "C.tar"
    assert [(i, h.hex()) for i, h in entries] == list(enumerate(C_DIGESTS))


def test_has_get_files_of_reference(bt):
    assert [(i, h.hex()) for i, h in bt.parse_chunk_list(os.path.join(GOLDEN, "ref_A.chunks"))] == \
        [(0, C_DIGESTS[0]), (1, C_DIGESTS[1])]
    assert [(i, h.hex()) for i, h in bt.parse_chunk_list(os.path.join(GOLDEN, "ref_B.chunks"))] == \
        [(2, C_DIGESTS[2]), (3, C_DIGESTS[3])]
    # make-chunks stdout is itself a valid has/get file
    got = bt.parse_chunk_list(os.path.join(GOLDEN, "C.tar.make-chunks.out"))
    assert [h.hex() for _, h in got] == C_DIGESTS


def test_generate_chunks_style_files(bt, tmp_path):
    # generate_chunks.py:5-18: 2000-line has files and a 4000-line master
    p1, pm = tmp_path / "1.haschunks", tmp_path / "master.haschunks"
    p1.write_text("".join(f"{i} {C_DIGESTS[2]}\n" for i in range(2000)))
    pm.write_text("File: NOEXIST.tar\nChunks:\n" + "".join(f"{i} {C_DIGESTS[2]}\n" for i in range(2000))
                  + "".join(f"{2000 + i} {C_DIGESTS[3]}\n" for i in range(2000)))
    e1 = bt.parse_chunk_list(p1)
    assert len(e1) == 2000 and e1[1999] == (1999, bytes.fromhex(C_DIGESTS[2]))
    name, em = bt.parse_master(pm)
    assert name == "NOEXIST.tar" and len(em) == 4000 and em[3999] == (3999, bytes.fromhex(C_DIGESTS[3]))


def test_comments_blank_and_malformed(bt, tmp_path):
    p = tmp_path / "x.chunks"
    p.write_text(f"# comment\n\n0 {C_DIGESTS[0]}\n# another\n7 {C_DIGESTS[1].upper()}\n")
    assert bt.parse_chunk_list(p) == [(0, bytes.fromhex(C_DIGESTS[0])), (7, bytes.fromhex(C_DIGESTS[1]))]
    for bad in [f"0 {C_DIGESTS[0][:-1]}\n", f"0 {C_DIGESTS[0]}x\n", f"0 {C_DIGESTS[0][:-1]}g\n", "zero abc\n",
                f"0 {C_DIGESTS[0]} trailing\n"]:
        p.write_text(f"1 {C_DIGESTS[1]}\n" + bad)
        with pytest.raises(bt.BtSha1Error, match=r"x.chunks:2"):
            bt.parse_chunk_list(p)
    with pytest.raises(bt.BtSha1Error, match="header"):
        bt.parse_master(os.path.join(GOLDEN, "ref_A.chunks"))
    with pytest.raises(bt.BtSha1Error, match="cannot open"):
        bt.parse_chunk_list(tmp_path / "missing")


def test_write_round_trip_matches_make_chunks_format(bt, tmp_path):
    d = [bytes.fromhex(h) for h in C_DIGESTS]
    p = tmp_path / "o.chunks"
    bt.write_chunks(p, d)
    assert p.read_text() == open(os.path.join(GOLDEN, "C.tar.make-chunks.out")).read()
    bt.write_chunks(p, d, master_name="C.tar")
    assert p.read_text() == open(os.path.join(GOLDEN, "ref_C.chunks")).read()
    bt.write_chunks(p, d[2:], first_id=2)
    assert p.read_text() == open(os.path.join(GOLDEN, "ref_B.chunks")).read()


def test_checked_hex(bt):
    assert bt.hex2binary_checked(C_DIGESTS[0]) == bytes.fromhex(C_DIGESTS[0])
    assert bt.hex2binary_checked(C_DIGESTS[0].upper()) == bytes.fromhex(C_DIGESTS[0])
    for bad in ["0g", "zz", "1", " 1"]:
        with pytest.raises(ValueError):
            bt.hex2binary_checked(bad)


CHUNKS_REF = os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "chunks-ref")


def _ref_table(mode, path):
    """The reference's own parser (util.c, compiled by oracle/Makefile) on a file."""
    import subprocess
    out = subprocess.run([CHUNKS_REF, mode, str(path)], capture_output=True, text=True, check=True).stdout.split("\n")
    n = int(out[0])
    return [(int(i), bytes.fromhex(h)) for i, h in (l.split() for l in out[1:1 + n])]


def _entries_and_text(data):
    """Well-formed .chunks bodies the reference parses without undefined
    behaviour: "<id><ws><40 hex>" lines, any hex case, spaces or tabs, LF or
    CRLF, the last line with or without its newline."""
    from hypothesis import strategies as st
    line = st.tuples(st.integers(-2**31, 2**31 - 1), st.binary(min_size=20, max_size=20),
                     st.sampled_from(["lower", "upper", "mixed"]), st.sampled_from([" ", "  ", "\t", " \t "]),
                     st.sampled_from(["\n", "\r\n", " \n"]))
    lines = data.draw(st.lists(line, min_size=0, max_size=60))
    text, entries = "", []
    for k, (i, h, case, ws, eol) in enumerate(lines):
        hx = h.hex()
        hx = hx.upper() if case == "upper" else (
            "".join(c.upper() if j % 2 else c for j, c in enumerate(hx)) if case == "mixed" else hx)
        text += f"{i}{ws}{hx}" + ("" if k == len(lines) - 1 and data.draw(st.booleans()) else eol)
        entries.append((i, h))
    return entries, text


@pytest.mark.skipif(not os.path.exists(CHUNKS_REF), reason="oracle/_ref/chunks-ref not built (no reference sources)")
def test_parsers_agree_with_the_reference_parsers(bt, tmp_path_factory):
    """Differential, property-based: libbtsha1's has/get and master parsers
    against the reference's parse_has_get_chunk_file / parse_total_chunk_file
    (util.c:64-164, compiled unmodified) on random well-formed files."""
    from hypothesis import given, settings, strategies as st

    @settings(max_examples=80, deadline=None)
    @given(st.data())
    def check(data):
        entries, body = _entries_and_text(data)
        d = tmp_path_factory.mktemp("fz")
        lst, master = d / "x.chunks", d / "m.chunks"
        lst.write_text(body)
        master.write_text("File: some.tar\nChunks:\n" + body)
        assert bt.parse_chunk_list(lst) == _ref_table("list", lst) == entries
        name, got = bt.parse_master(master)
        assert name == "some.tar" and got == _ref_table("master", master) == entries
    check()
