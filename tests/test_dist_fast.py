"""The multi-rank build's fused leaf + layer-0 schedule (gcz_dist_fast.h, gcz_group::build_fast).

Layer 0 is hash-consed across ranks with the leaves' hashed codes as labels, in the same
collective groups as the leaf-id exchange; the layer-0 nodes are canonicalised with the global
leaf ids only afterwards.  Its trees must equal the reference's (goldens) and the general
schedule's (GCZ_DIST_FAST=0) byte for byte; inputs it does not cover (IUPAC, repetitive data,
a layer 1 that is not direct, C/D slot overflows) must fall back to the general schedule with
the same result.  Virtual ranks on one MI355X (gcz_group_create_local).
"""
import os

import numpy as np
import pytest

from conftest import case_input, compare_digest

pytestmark = pytest.mark.gpu


def _group(gcz, world, env=None):
    env = env or {}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return gcz.Group.local(world)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _build(gcz, g, bases, L=12):
    S = len(bases) // L
    ctx0 = g.ctx(0)
    buf = ctx0.upload(np.frombuffer(bases, np.uint8) if isinstance(bases, bytes) else bases)
    try:
        ptrs = [buf.ptr + gcz.dist_plan(S, g.world, r)[0] * L for r in range(g.world)]
        return g.build_device_bases(ptrs, S, L)
    finally:
        buf.free()


def _schedule(g):
    """'fast' / 'general' / 'fast, discarded' from the last build's exchange log."""
    names = [e["name"] for e in g.exchange_log(0)]
    fast = any(n.startswith("R1a ") for n in names)
    general = any(n in ("keys to owners", "leaf presence bitmaps + status") for n in names)
    return "fast, discarded" if fast and general else "fast" if fast else "general"


def _single(gcz, bases, L=12):
    c = gcz.Context(0)
    try:
        c.build_fasta(b">x\n" + bytes(bases) + b"\n", L)
        return gcz.digest(c.tree())
    finally:
        c.close()


@pytest.fixture(scope="module")
def uniform_100m(gcz, manifest):
    case = manifest["synth/uniform_100000003"]
    kind, payload, L = case_input(case, gcz)
    return np.frombuffer(gcz.fasta_extract(payload, L), np.uint8).copy(), case["expect"]


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("tail", ["9", None])
def test_fast_schedule_uniform_golden(world, tail, gcz, uniform_100m, monkeypatch):
    """100 Mbase uniform ACGT: the fused schedule is taken (9 collective groups, K2 on the bulk stream) and the tree
    equals the compiled reference's, at the deep and at the default partition depth."""
    if tail:
        monkeypatch.setenv("GCZ_DIST_TAIL_LOG2", tail)
    bases, exp = uniform_100m
    g = _group(gcz, world)
    try:
        _build(gcz, g, bases)
        assert _schedule(g) == "fast"
        log = g.exchange_log(0)
        assert len(log) == 9, [e["name"] for e in log]
        assert compare_digest(gcz.digest(g.tree()), exp) == {}
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 5, 8])
def test_fast_equals_general_random(world, gcz):
    """Random ACGT genomes (odd strand counts: the null pair at the end) -- fused schedule,
    general schedule and one-device build byte-identical."""
    rng = np.random.default_rng(world)
    for nbases in (24_000_012, 30_000_000 + 12 * 7):
        bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=nbases)].copy()
        ref = _single(gcz, bases)
        got = {}
        for mode in ("1", "0"):
            g = _group(gcz, world, {"GCZ_DIST_FAST": mode})
            try:
                _build(gcz, g, bases)
                got[mode] = (_schedule(g), gcz.digest(g.tree()))
            finally:
                g.close()
        assert got["1"][0] == "fast" and got["0"][0] == "general", (got["1"][0], got["0"][0])
        assert got["1"][1] == ref, (world, nbases)
        assert got["0"][1] == ref, (world, nbases)


def _with_repeats(rng, nbases, L, block, every_other):
    """Uniform ACGT with repeated layer-0 pairs: a copied block of `block` strands (whole pairs
    and layer-1 pairs repeat: layer 1 is not direct), or every other pair of a region copied
    (many repeated layer-0 pairs, but no layer-1 pair with two repeated children)."""
    strands = rng.integers(0, 4, size=(nbases // L, L), dtype=np.uint8)
    S = strands.shape[0]
    if every_other:
        src = np.arange(0, S // 3, 4)                       # pairs (2j, 2j+1) with j even
        dst = src + (S // 2 // 4) * 4
        strands[dst] = strands[src]
        strands[dst + 1] = strands[src + 1]
    else:
        strands[S // 2:S // 2 + block] = strands[16:16 + block]
    return np.frombuffer(b"ACGT", np.uint8)[strands].reshape(-1).copy()


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("shape", ["block", "every_other"])
def test_fast_discards_and_falls_back(world, shape, gcz):
    """A copied region (layer 1 not direct) or thousands of cross-rank repeats of layer-0
    pairs (C slots overflow): every rank discards the fused attempt after its final vectors and
    the general schedule builds the same tree as one device."""
    rng = np.random.default_rng(100 + world)
    bases = _with_repeats(rng, 36_000_000, 12, 16_384, shape == "every_other")
    ref = _single(gcz, bases)
    g = _group(gcz, world)
    try:
        _build(gcz, g, bases)
        assert _schedule(g) == "fast, discarded"
        assert gcz.digest(g.tree()) == ref
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 8])
def test_fast_owner_region_overflow_falls_back(world, gcz, monkeypatch):
    """Owner regions of the keys' scatter (k_fl_scatter) too small for their records: the surplus
    is dropped in bounds, status bit 4 reaches every rank in R1a, and the general schedule
    builds the same tree as one device."""
    monkeypatch.setenv("GCZ_FL_CAP_PERMILLE", "900")
    rng = np.random.default_rng(300 + world)
    bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=24_000_000 + 12 * 3)].copy()
    ref = _single(gcz, bases)
    g = _group(gcz, world)
    try:
        _build(gcz, g, bases)
        assert _schedule(g) == "fast, discarded"
        assert gcz.digest(g.tree()) == ref
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 4])
def test_fast_declines_repetitive_and_iupac(world, gcz, manifest):
    """Inputs outside the fused schedule decide at the mid-build read (R1's status words):
    tandem repeats (repetitive data) and a genome with an IUPAC code -- the general schedule
    runs from there and matches the reference / one device."""
    case = manifest["synth/tandem_100000000"]
    kind, payload, L = case_input(case, gcz)
    bases = np.frombuffer(gcz.fasta_extract(payload, L), np.uint8).copy()
    g = _group(gcz, world)
    try:
        _build(gcz, g, bases)
        assert _schedule(g) == "fast, discarded"
        assert compare_digest(gcz.digest(g.tree()), case["expect"]) == {}
        rng = np.random.default_rng(7)
        iu = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=24_000_000)].copy()
        iu[23_000_005] = ord("R")
        _build(gcz, g, iu)
        assert _schedule(g) == "fast, discarded"
        assert gcz.digest(g.tree()) == _single(gcz, iu)
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_fast_equals_general_symmetric_variants(world, gcz):
    """Pairs next to their symmetric variants: (A, B) with (A mirrored, B), (A transposed, B),
    (A, B mirrored), the mirrored node (B~, A~), the transposed node (A', B') and palindromic
    leaves -- every child bit the 6-byte records re-label (canonical-code rank, m, t) must keep
    distinct classes apart and equal ones together."""
    rng = np.random.default_rng(40 + world)
    L = 12
    comp = np.array([3, 2, 1, 0], np.uint8)      # A<->T, C<->G on codes 0..3 = A,C,G,T
    base = rng.integers(0, 4, size=(1_000_000, L), dtype=np.uint8)
    pal = base[:1000, :6]
    base[:1000] = np.concatenate([pal, pal[:, ::-1]], axis=1)   # mirror-invariant leaves
    a, b = base[0::2], base[1::2]
    variants = [(a, b), (a[:, ::-1], b), (comp[a], b), (a, b[:, ::-1]), (b[:, ::-1], a[:, ::-1]),
                (comp[a], comp[b]), (comp[b][:, ::-1], comp[a][:, ::-1]), (a, comp[b])]
    pairs = []
    for x, y in variants:
        pairs.append(np.stack([x, y], axis=1))
    strands = np.concatenate(pairs).reshape(-1, L)
    order = rng.permutation(strands.shape[0] // 2)
    strands = strands.reshape(-1, 2, L)[order].reshape(-1, L)
    bases = np.frombuffer(b"ACGT", np.uint8)[strands].reshape(-1).copy()
    ref = _single(gcz, bases)
    g = _group(gcz, world)
    try:
        _build(gcz, g, bases)
        assert _schedule(g) in ("fast", "fast, discarded")
        assert gcz.digest(g.tree()) == ref
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 8])
def test_fast_schedule_bulk_second_stream(world, gcz, uniform_100m):
    """K2 on a real second stream (GCZ_LOCAL_BULK=1: the local transport's bulk copies run
    there, ordered only by the schedule's ev_bulk_in / ev_bulk_out, as RCCL's communicator 2
    runs them): the tree equals the reference's, and a discarded attempt after K2 (a copied
    block: layer 1 not direct) falls back to the same tree as one device."""
    bases, exp = uniform_100m
    g = _group(gcz, world, {"GCZ_LOCAL_BULK": "1"})
    try:
        assert g.has_bulk
        for _ in range(2):   # (the second build reuses the events and buffers)
            _build(gcz, g, bases)
            names = [e["name"] for e in g.exchange_log(0)]
            assert _schedule(g) == "fast" and len(names) == 9, names
            assert any("second stream" in n for n in names), names
            assert compare_digest(gcz.digest(g.tree()), exp) == {}
        rng = np.random.default_rng(500 + world)
        rep = _with_repeats(rng, 24_000_000, 12, 16_384, False)
        _build(gcz, g, rep)
        assert _schedule(g) == "fast, discarded"
        assert gcz.digest(g.tree()) == _single(gcz, rep)
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("cap", ["0", "1"])
def test_fast_lookback_give_up(world, cap, gcz, uniform_100m, monkeypatch):
    """k_fl_scatter's look-back gives up (GCZ_FL_SPIN_CAP; 0: every tile after the first at
    once): the tile publishes a partial prefix and sets status bit 256, the records it misplaces
    stay inside their regions, every rank runs the general schedule and the tree equals the
    reference's.  cap 1: whichever tiles happen to give up -- the same tree either way."""
    monkeypatch.setenv("GCZ_FL_SPIN_CAP", cap)
    bases, exp = uniform_100m
    g = _group(gcz, world)
    try:
        _build(gcz, g, bases)
        if cap == "0":
            assert _schedule(g) == "fast, discarded"
        assert compare_digest(gcz.digest(g.tree()), exp) == {}
    finally:
        g.close()


@pytest.mark.parametrize("L", [8, 9, 11])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_fast_equals_general_other_L(L, world, gcz):
    """Strand lengths other than 12: Bc = 2L - 1 code bits, the 6-byte record's key bits, the
    relay slots' bound (canonical orbits of 2L-bit codes) and small bucket words -- fused
    schedule, general schedule and one device byte-identical."""
    rng = np.random.default_rng(1000 * L + world)
    nbases = 12_000_000 // L * L + L * 5
    bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=nbases)].copy()
    ref = _single(gcz, bases, L)
    got = {}
    for mode in ("1", "0"):
        g = _group(gcz, world, {"GCZ_DIST_FAST": mode})
        try:
            _build(gcz, g, bases, L)
            got[mode] = (_schedule(g), gcz.digest(g.tree()))
        finally:
            g.close()
    assert got["0"][0] == "general"
    assert got["1"][0] == "fast" if L >= 9 else got["1"][0] in ("fast", "fast, discarded"), got["1"][0]
    assert got["1"][1] == ref, (L, world)
    assert got["0"][1] == ref, (L, world)


@pytest.mark.parametrize("world,tail", [(2, "9"), (2, None), (3, "9"), (8, "9"), (8, None)])
def test_fast_schedule_guard_bands(world, tail, gcz, uniform_100m, monkeypatch):
    """No kernel of the fused schedule stores past a buffer (GCZ_CANARY=1: a 4 KB guard band
    after every buffer the library sizes, checked after each build), at the shape of round 5's
    illegal accesses (world 2, GCZ_DIST_TAIL_LOG2=9: rank 0's level buffers sized by its own
    3.5 M strands instead of the whole genome) and around it; first build of fresh contexts
    (every buffer allocated by that build) and a second one."""
    if tail:
        monkeypatch.setenv("GCZ_DIST_TAIL_LOG2", tail)
    bases, exp = uniform_100m
    g = _group(gcz, world, {"GCZ_CANARY": "1"})
    try:
        for _ in range(2):
            _build(gcz, g, bases)
            assert _schedule(g) == "fast"
            assert g.canary_check() == ""
        assert compare_digest(gcz.digest(g.tree()), exp) == {}
        rng = np.random.default_rng(77)
        rep = _with_repeats(rng, 24_000_000, 12, 16_384, True)   # discarded: the general schedule too
        _build(gcz, g, rep)
        assert g.canary_check() == ""
    finally:
        g.close()


def test_single_device_guard_bands(gcz, manifest):
    """The one-device build (dense leaf level, bucketed layer 0, direct subtrees, tail; tandem:
    the hash-table levels with the block pre-dedupe) stores nothing past its buffers."""
    os.environ["GCZ_CANARY"] = "1"
    try:
        c = gcz.Context(0)
    finally:
        del os.environ["GCZ_CANARY"]
    try:
        assert gcz._lib.gcz_ctx_canary_selftest(c._h) == 0   # (the check sees a planted overwrite)
        for name in ("synth/uniform_100000003", "synth/tandem_100000000", "corpus/merged"):
            case = manifest[name]
            kind, payload, L = case_input(case, gcz)
            c.build_fasta(payload, L)
            assert c.canary_check() == "", name
            assert compare_digest(gcz.digest(c.tree()), case["expect"]) == {}, name
    finally:
        c.close()
