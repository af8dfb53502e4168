"""Reader buffers that are not a power of two: shared_tree{fasta_reader{path, B}}.

The reference reduces every fasta_reader buffer of B strands to its own subtree -- pairing
inside the buffer, an odd buffer's last element with null -- and then combines the roots
(src/shared_tree.cpp:719-736, reduce_segment include/shared_tree.h:305-316).  For the default
reader (power-of-two buffers) that is the global level loop; for other B the device build
expands each level's input with a null after every odd buffer (k_seg_expand, gcz_device.h).
Pinned by the compiled reference's segbuf/ goldens (tests/golden/make_goldens.py
--segmented) and by the oracle's restatement of the buffer loop on random inputs.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_input, compare_digest

pytestmark = pytest.mark.gpu


def _segbuf_names():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        m = json.load(f)
    return [n for n, c in sorted(m.items()) if "buffer" in c]


def _ctx_env(gcz, env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return gcz.Context(0)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module", params=[{}, {"GCZ_BUCKET_MIN": "1"}, {"GCZ_DENSE": "2", "GCZ_TABLE": "wide"}],
            ids=["default", "bucketed", "dense-wide"])
def ctx_seg(request, gcz):
    c = _ctx_env(gcz, request.param)
    yield c
    c.close()


@pytest.mark.parametrize("name", _segbuf_names())
def test_gpu_reader_buffers_match_reference(name, ctx_seg, gcz, manifest):
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    if exp["exit"] != 0:
        with pytest.raises(gcz.GczError) as ei:
            ctx_seg.build_fasta_buffered(payload, L, case["buffer"])
        assert ei.value.code == gcz.GCZ_ERR_SYMBOL
        return
    info = ctx_seg.build_fasta_buffered(payload, L, case["buffer"])
    assert info["layer_size"] == exp["layer_sizes"]
    assert compare_digest(gcz.digest(ctx_seg.tree()), exp) == {}
    ctx_seg.sort_device()
    assert hashlib.sha256(ctx_seg.serialize_device()).hexdigest() == exp["sha_dag"]


def test_gpu_reader_buffers_random(gcz, oracle):
    """Random genomes (pure ACGT and IUPAC, repeat-heavy and unique) at random buffer sizes,
    and readers whose first buffers were already read out, against the oracle."""
    ctx = gcz.Context(0)
    rng = np.random.default_rng(41)
    try:
        for trial in range(24):
            L = int(rng.choice([1, 3, 12, 16]))
            S = int(rng.integers(2, 60_000))
            alphabet = np.frombuffer(b"ACGT" if trial % 3 else b"ACGTNRYacgt", dtype=np.uint8)
            if trial % 4 == 0:   # repeats: a small pool of strands
                pool = alphabet[rng.integers(0, alphabet.size, size=(8, L))]
                bases = pool[rng.integers(0, 8, size=S)].reshape(-1)
            else:
                bases = alphabet[rng.integers(0, alphabet.size, size=S * L)]
            data = bases.tobytes()
            B = int(rng.integers(1, max(2, S)))
            nseg = (S + B - 1) // B
            first = B * int(rng.integers(0, nseg)) if trial % 5 == 0 else 0
            ctx.build_fasta_buffered(data, L, B, first)
            g = ctx.tree()
            o = oracle.build_fasta_buffered(data, L, B, first)
            ctx_info = (trial, L, S, B, first)
            assert g.leaves_bin() == o.leaves_bin(), ctx_info
            assert g.layers_bin() == o.layers_bin(), ctx_info
            assert g.root == o.root, ctx_info
    finally:
        ctx.close()


def test_gpu_reader_power_of_two_is_global(gcz, manifest):
    """A power-of-two buffer of >= 2 strands (the reference default 2^22 included) gives the
    global tree (buffers of one strand do not: segbuf/chmpxx_L12_B1)."""
    ctx = gcz.Context(0)
    try:
        with open(os.path.join(GOLDEN, "data", "chmpxx"), "rb") as f:
            data = f.read()
        exp = manifest["corpus/chmpxx"]["expect"]
        for B in (2, 64, 1024, 1 << 22, 0):
            ctx.build_fasta_buffered(data, 12, B)
            assert compare_digest(gcz.digest(ctx.tree()), exp) == {}, B
    finally:
        ctx.close()


def test_gpu_reader_all_buffers_read(gcz):
    """A reader whose every buffer was already handed out (read_into) leaves no strand to
    build: the reference reduces an empty root list (undefined); here a clear GCZ_ERR_ARG
    naming it, and the context builds normally afterwards.  (Parity unpinned: no reference
    output exists for this case.)"""
    ctx = gcz.Context(0)
    try:
        data = b"ACGT" * 3000          # 1000 strands of 12
        for B, first in ((100, 1000), (256, 1024), (7, 1001)):
            with pytest.raises(gcz.GczError) as ei:
                ctx.build_fasta_buffered(data, 12, B, first)
            assert ei.value.code == gcz.GCZ_ERR_ARG
            assert "already read" in str(ei.value)
        info = ctx.build_fasta_buffered(data, 12, 100, 900)
        assert info["n_strands"] == 100
    finally:
        ctx.close()
