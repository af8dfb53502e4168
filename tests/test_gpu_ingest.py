"""FASTA ingest on the device against the reference reader's
line contract (src/fasta_reader.cpp:40-68; host restatement gcz_fasta_extract and
the C oracle) and the goldens built by the compiled reference."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_input, compare_digest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(gcz):
    c = gcz.Context(0)
    yield c
    c.close()


EDGE = [b"", b"\n", b"\n\n", b">h\n", b">h", b"ACGT", b"ACGT\n", b"ACGT\n\n", b">h\nACGT\n>h2\nTTGA",
        b">a\n>b\nACGT\n", b"\n>x\nAC\n", b">a\n\nGG\n", b"\n\n\n\nAC\n", b">1\n>2\n>3\n>4\nA\n",
        b"AC\r\nGT\r\n", b"A" * 5000 + b"\n" + b"C" * 3000, b"\n".join([b"ACGTN"] * 3000), b">" * 10 + b"\nAC"]


@pytest.mark.parametrize("i", range(len(EDGE)))
def test_device_extract_edge_cases(i, ctx, gcz, oracle):
    data = EDGE[i]
    assert ctx.fasta_extract_device(data) == gcz.fasta_extract(data) == oracle.fasta_extract(data)


def test_device_extract_random_line_soup(ctx, gcz):
    rng = np.random.default_rng(3)
    for trial in range(20):
        lines = []
        for _ in range(int(rng.integers(1, 4000))):
            r = rng.random()
            if r < 0.15:
                lines.append(b">hdr" + bytes(rng.integers(65, 90, size=int(rng.integers(0, 20))).astype(np.uint8)))
            elif r < 0.25:
                lines.append(b"")
            else:
                lines.append(bytes(rng.choice(np.frombuffer(b"ACGTacgtN", np.uint8), size=int(rng.integers(1, 300)))))
        data = b"\n".join(lines) + (b"\n" if trial % 2 else b"")
        assert ctx.fasta_extract_device(data) == gcz.fasta_extract(data), trial


def _fasta_cases():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        m = json.load(f)
    return [n for n, c in sorted(m.items()) if c["kind"] == "fasta" and "buffer" not in c]


@pytest.mark.parametrize("name", _fasta_cases())
def test_device_fasta_build_matches_reference(name, ctx, gcz, manifest):
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    buf = ctx.upload(np.frombuffer(payload, dtype=np.uint8) if payload else np.zeros(1, np.uint8))
    try:
        if exp["exit"] != 0:
            with pytest.raises(gcz.GczError) as ei:
                ctx.build_device_fasta(buf.ptr, len(payload), L)
            if ei.value.code == gcz.GCZ_ERR_SYMBOL:
                sym = ei.value.info["error_symbol"]
                sym = sym - 32 if 97 <= sym <= 122 else sym
                assert f"Encountered unknown symbol: {sym} (ASCII code {sym})" == exp["stderr"]
            return
        ctx.build_device_fasta(buf.ptr, len(payload), L)
    finally:
        buf.free()
    assert compare_digest(gcz.digest(ctx.tree()), exp) == {}


# ---- reader buffers (src/fasta_reader.cpp:22-31,47-64; tests/test_reader_boundary.py) ----
def test_device_reader_cases_match_reference(ctx, oracle):
    """The device ingest at reader buffers of 1-8 strands == the compiled reference's strands."""
    with open(os.path.join(GOLDEN, "reader_cases.json")) as f:
        cases = json.load(f)
    for i, c in enumerate(cases):
        data, L, buf = bytes.fromhex(c["input_hex"]), c["L"], c["buffer"]
        bases = ctx.fasta_extract_device(data, L, buf)
        assert bases == oracle.fasta_extract(data, L, buf), (i, data, L, buf)
        try:
            got = [int(v) for v in oracle.pack(bases, L)]
        except oracle.OracleError as e:
            got = str(e)
        exp = c["expect"]["strands"] if c["expect"]["exit"] == 0 else c["expect"]["stderr"]
        assert got == exp, (i, data, L, buf)


def _big_cases():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        m = json.load(f)
    return [n for n, c in sorted(m.items()) if c["kind"] == "fastabig"]


@pytest.mark.parametrize("name", _big_cases())
def test_device_fasta_big_matches_reference(name, ctx, gcz, manifest):
    """~100 MB wrapped multi-record FASTA over two reader buffers (headers, blank
    lines, '>' at the boundaries), uploaded and built like shared_tree{path}."""
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    if exp["exit"] != 0:
        with pytest.raises(gcz.GczError) as ei:
            ctx.build_fasta(payload, L)
        assert ei.value.code == gcz.GCZ_ERR_SYMBOL
        sym = ei.value.info["error_symbol"]
        sym = sym - 32 if 97 <= sym <= 122 else sym
        assert f"Encountered unknown symbol: {sym} (ASCII code {sym})" == exp["stderr"]
        return
    ctx.build_fasta(payload, L)
    assert compare_digest(gcz.digest(ctx.tree()), exp) == {}
