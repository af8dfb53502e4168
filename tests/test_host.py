"""libgcz host-side entry points (no GPU): C ABI exports, FASTA contract,
frequency sort / bytes / serialize / width / deserialize, synthetic generator."""
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, REPO, case_input, compare_digest


def header_symbols():
    with open(os.path.join(REPO, "include", "gcz.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"GCZ_API\s+[\w\s\*]*?\b(gcz_\w+)\s*\(", text)))


def test_abi_exports_every_declared_symbol(gcz):
    import ctypes
    syms = header_symbols()
    assert len(syms) >= 38
    lib = ctypes.CDLL(gcz.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert missing == []
    # the Python binding wraps every declared entry point
    assert sorted(set(gcz.EXPORTED)) == syms


def test_host_storage_pool(gcz):
    """The containers' host storage (gcz_host_alloc / free / prefault / pool_release): small
    arrays from the heap, large ones as 2 MB-aligned mappings, carved from a pre-faulted pool
    while it lasts, then mapped fresh; every piece unmaps alone."""
    import ctypes
    lib = gcz._lib
    MB = 1 << 20
    assert lib.gcz_host_prefault(64 * MB, 4) == 0
    pieces = []
    for nbytes in (1000, 5 * MB, 17 * MB + 3, 30 * MB, 40 * MB):   # the last one exceeds the pool's rest
        p = lib.gcz_host_alloc(nbytes)
        assert p
        if nbytes >= 4 * MB:
            assert p % (2 * MB) == 0
        ctypes.memset(p, 0x5A, nbytes)
        pieces.append((p, nbytes))
    big = [p for p, n in pieces if n >= 4 * MB]
    assert big[1] == big[0] + 6 * MB and big[2] == big[1] + 18 * MB   # carved back to back from the pool
    for p, nbytes in pieces:
        assert ctypes.string_at(p + nbytes - 1, 1) == b"Z"
        lib.gcz_host_free(p, nbytes)
    lib.gcz_host_pool_release(0)
    lib.gcz_host_pool_release(1)   # (idempotent; async)
    assert lib.gcz_host_prefault(8 * MB, 2) == 0
    lib.gcz_host_pool_release(1)


def test_fasta_extract_matches_oracle(gcz, oracle, manifest):
    for name, case in manifest.items():
        if case["kind"] != "fasta":
            continue
        with open(os.path.join(GOLDEN, case["input"]), "rb") as f:
            data = f.read()
        assert gcz.fasta_extract(data, case["L"]) == oracle.fasta_extract(data, case["L"]), name


@pytest.mark.parametrize("name", ["corpus/chmpxx", "corpus/hehcmv", "corpus/merged", "corpus/edited",
                                  "fasta/iupac_stress", "vectors/ref_frequency_sort", "vectors/pool_S4097",
                                  "vectors/L16_edges_S5000", "lsweep/chmpxx_L1", "lsweep/chmpxx_L16",
                                  "synth/tandem_10000000"])
def test_host_tree_ops_match_reference(name, gcz, oracle, manifest):
    """Build with the oracle, hand the unsorted tree to libgcz, and check libgcz's
    sort_tree / bytes / serialize / width against the reference goldens."""
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    ot = oracle.build_fasta(payload, L) if kind == "fasta" else oracle.build_leaves(payload, L)
    t = gcz.Tree.from_arrays(L, ot.leaves(), [ot.layer(k) for k in range(ot.n_layers)], ot.root)
    assert compare_digest(gcz.digest(t), case["expect"]) == {}


def test_deserialize_roundtrip(gcz, oracle):
    import gzip
    with gzip.open(os.path.join(GOLDEN, "full", "hehcmv.dag.gz")) as f:
        dag = f.read()
    t = gcz.Tree.deserialize(dag, 12)
    assert t.serialize() == dag
    assert t.width() == 19112
    # invariant bits are not stored on disk (pointer::deserialize, shared_tree.cpp:147-163)
    assert all((t.layer(k) >> 31).max() == 0 for k in range(t.n_layers))


def test_deserialize_rejects_truncated(gcz):
    with pytest.raises(gcz.GczError):
        gcz.Tree.deserialize(b"\x00\x00\x00", 12)


def test_synth_is_deterministic_and_random_access(gcz):
    a = gcz.synth(0, 1000)
    assert set(a.tobytes()) <= set(b"acgt")
    b = gcz.synth(0, 5000)
    assert (b[:1000] == a).all()
    t = gcz.synth(1, 300_000)
    assert set(t.tobytes()) <= set(b"acgt")
    # tandem genome really repeats: many identical 12-mers
    k = np.frombuffer(t.tobytes()[: 12 * 20000], dtype="S12")
    assert len(set(k.tolist())) < 0.9 * len(k)
