"""The C restatement (oracle/) pinned against the compiled reference's golden vectors."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_input, compare_digest

SMALL_CASES = None


def _cases(manifest, max_bases=12_000_000):
    out = []
    for name, case in sorted(manifest.items()):
        if (case["kind"] == "synth" and case["nbases"] > max_bases) or case["kind"] == "fastabig":
            continue
        out.append(name)
    return out


def pytest_generate_tests(metafunc):
    if "oracle_case" in metafunc.fixturenames:
        import json
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            m = json.load(f)
        metafunc.parametrize("oracle_case", _cases(m))


def test_oracle_matches_reference(oracle_case, manifest, oracle, gcz):
    case = manifest[oracle_case]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    buf = case.get("buffer")   # segbuf/: reader buffers of B strands, each its own subtree
    if exp["exit"] != 0:
        with pytest.raises(oracle.OracleError) as ei:
            oracle.build_fasta(payload, L) if buf is None else oracle.build_fasta_buffered(payload, L, buf)
        assert str(ei.value) == exp["stderr"]
        return
    if buf is not None:
        tree = oracle.build_fasta_buffered(payload, L, buf)
    else:
        tree = oracle.build_fasta(payload, L) if kind == "fasta" else oracle.build_leaves(payload, L)
    got = oracle.digest(tree)
    assert compare_digest(got, exp) == {}


def test_oracle_full_dump_chmpxx(oracle):
    import gzip
    with open(os.path.join(GOLDEN, "data", "chmpxx"), "rb") as f:
        t = oracle.build_fasta(f.read(), 12)
    with gzip.open(os.path.join(GOLDEN, "full", "chmpxx.leaves.bin.gz")) as f:
        assert t.leaves_bin() == f.read()
    with gzip.open(os.path.join(GOLDEN, "full", "chmpxx.layers.bin.gz")) as f:
        assert t.layers_bin() == f.read()


def test_leaf_codec_known_answers(oracle):
    # tests/test.cpp:33-45: transposed(AAAA..) == TTTT..; mirrored reverses
    lib = oracle.lib
    A = int("".join(["1"] * 12), 16)     # nibble 1 = A
    T = int("".join(["8"] * 12), 16)     # nibble 8 = T
    assert lib.orc_leaf_transposed(A) == T
    p = oracle.pack(b"ACTGACTGACTG", 12)[0]
    q = oracle.pack(b"GTCAGTCAGTCA", 12)[0]
    assert lib.orc_leaf_mirrored(int(p), 12) == int(q)


def test_pointer_known_answers(oracle):
    # tests/test.cpp:47-59
    lib = oracle.lib
    basis = 3280
    assert lib.orc_ptr_xf(basis, 0, 1) != basis
    assert lib.orc_ptr_xf(basis, 1, 0) != basis
    null = 0x9FFFFFFF
    assert lib.orc_ptr_xf(null, 1, 1) == null


def test_node_canonical_invariance(oracle):
    # tests/test.cpp:117-129: canonical(node) is invariant under mirror/transpose/invert
    import ctypes
    lib = oracle.lib

    def canon(l, r):
        cl, cr = ctypes.c_uint32(), ctypes.c_uint32()
        m, t = ctypes.c_int(), ctypes.c_int()
        lib.orc_node_canonical(l, r, ctypes.byref(cl), ctypes.byref(cr), ctypes.byref(m), ctypes.byref(t))
        return cl.value & 0x7FFFFFFF, cr.value & 0x7FFFFFFF

    xf = lib.orc_ptr_xf
    rng = np.random.default_rng(3)
    for _ in range(200):
        l = int(rng.integers(0, 1 << 20)) | (int(rng.integers(0, 2)) << 29) | (int(rng.integers(0, 2)) << 30)
        r = int(rng.integers(0, 1 << 20)) | (int(rng.integers(0, 2)) << 30)
        a = canon(l, r)
        assert canon(xf(r, 1, 0), xf(l, 1, 0)) == a
        assert canon(xf(l, 0, 1), xf(r, 0, 1)) == a
        assert canon(xf(r, 1, 1), xf(l, 1, 1)) == a
