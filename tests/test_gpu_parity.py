"""Parity of the HIP build (libgcz, gfx950) with the compiled reference's goldens
and with the C oracle.  Every test here runs the MI355X kernels through the C ABI."""
import gzip
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


@pytest.fixture(scope="module")
def ctx_wide(gcz):
    """A context forced onto the 16-B wide table (the fallback path)."""
    os.environ["GCZ_TABLE"] = "wide"
    try:
        c = gcz.Context(0)
    finally:
        del os.environ["GCZ_TABLE"]
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_bucket(gcz):
    """A context that takes the bucketed LDS node insert on every hashed level."""
    os.environ["GCZ_BUCKET_MIN"] = "1"
    try:
        c = gcz.Context(0)
    finally:
        del os.environ["GCZ_BUCKET_MIN"]
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_bucket_rep(gcz):
    """The two-pass bucketed insert on every hashed level with the repetitive-data block
    collapse forced on (k_bkt_part: repeats inside 1024-pair blocks collapse, kNfDup)."""
    os.environ.update({"GCZ_BUCKET_MIN": "1", "GCZ_PREDUP": "1"})
    try:
        c = gcz.Context(0)
    finally:
        del os.environ["GCZ_BUCKET_MIN"], os.environ["GCZ_PREDUP"]
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_dense(gcz):
    """A context that runs the dense leaf level (gcz_dense.h) at every size."""
    os.environ["GCZ_DENSE"] = "2"
    try:
        c = gcz.Context(0)
    finally:
        del os.environ["GCZ_DENSE"]
    yield c
    c.close()


def _names(max_bases):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        m = json.load(f)
    return [n for n, c in sorted(m.items())
            if not (c["kind"] == "synth" and c["nbases"] > max_bases) and c["kind"] != "fastabig"
            and "buffer" not in c]


def _build(ctx, kind, payload, L):
    return ctx.build_fasta(payload, L) if kind == "fasta" else ctx.build_leaves(payload, L)


@pytest.mark.parametrize("name", [n for n in _names(12_000_000) if not n.startswith("fasta/")])
def test_gpu_bucketed_insert_goldens(name, ctx_bucket, gcz, manifest):
    """The bucketed node insert (k_bkt_*, forced on every hashed level) builds the
    reference's tree bit for bit."""
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    _build(ctx_bucket, kind, payload, L)
    assert compare_digest(gcz.digest(ctx_bucket.tree()), case["expect"]) == {}


@pytest.mark.parametrize("name", [n for n in _names(12_000_000) if not n.startswith("fasta/")])
def test_gpu_bucketed_collapse_goldens(name, ctx_bucket_rep, gcz, manifest):
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    info = _build(ctx_bucket_rep, kind, payload, L)
    assert compare_digest(gcz.digest(ctx_bucket_rep.tree()), case["expect"]) == {}
    if info["hashed_pairs"]:
        assert info["attempts"] == 1   # (no bucket overflow: hot keys collapse, big buckets loop)


def test_gpu_bucketed_collapse_random(ctx_bucket_rep, gcz, oracle):
    """Block collapse + looping dedupe on random leaf mixes from all-unique to a few hot keys
    (the hot keys fill buckets far beyond the register batch), against the oracle."""
    rng = np.random.default_rng(13)
    for S, pool_div in [(5, 1), (4097, 1), (100_003, 7), (300_001, 50_000), (400_000, 200_000),
                        (262_144, 4), (1_000_003, 333_334)]:
        pool = rng.integers(0, 1 << 48, size=max(4, S // pool_div), dtype=np.uint64)
        leaves = pool[rng.integers(0, pool.size, size=S)]
        ctx_bucket_rep.build_leaves(leaves, 12)
        g = ctx_bucket_rep.tree()
        o = oracle.build_leaves(leaves, 12)
        assert g.leaves_bin() == o.leaves_bin(), S
        assert g.layers_bin() == o.layers_bin(), S


@pytest.mark.parametrize("name", _names(12_000_000))
def test_gpu_dense_leaf_goldens(name, ctx_dense, gcz, manifest):
    """The dense leaf level forced at every size: pure-ACGT inputs with L <= 12 take
    it, every other input falls back to the hash-table level; both give the
    reference's tree bit for bit."""
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    if exp["exit"] != 0:
        with pytest.raises(gcz.GczError):
            _build(ctx_dense, kind, payload, L)
        return
    info = _build(ctx_dense, kind, payload, L)
    assert compare_digest(gcz.digest(ctx_dense.tree()), exp) == {}
    if name.startswith("synth/"):
        assert info["leaf_path"] == 1


def test_gpu_dense_leaf_random_acgt(ctx_dense, gcz, oracle):
    """Pure-ACGT leaves at every L <= 12 and sizes around the 32 Ki-strand chunks."""
    rng = np.random.default_rng(11)
    acgt = np.array([1, 2, 4, 8], dtype=np.uint64)
    for L, S in [(12, 1), (12, 2), (12, 1023), (12, 32767), (12, 32768), (12, 32769), (12, 100_003),
                 (11, 70_001), (10, 65_536), (9, 5_000), (8, 40_000), (7, 3_001), (6, 777), (5, 64), (4, 4097),
                 (3, 100), (2, 33), (1, 9), (12, 262_147)]:
        pool = rng.integers(0, 4, size=(max(2, S // 3), L))
        vals = (acgt[pool] << (4 * np.arange(L, dtype=np.uint64))).sum(axis=1).astype(np.uint64)
        leaves = vals[rng.integers(0, vals.size, size=S)]
        info = ctx_dense.build_leaves(leaves, L)
        assert info["leaf_path"] == 1, (L, S)
        g = ctx_dense.tree()
        o = oracle.build_leaves(leaves, L)
        assert g.leaves_bin() == o.leaves_bin(), (L, S)
        assert g.layers_bin() == o.layers_bin(), (L, S)
        assert g.root == o.root, (L, S)


@pytest.mark.parametrize("name", _names(12_000_000))
def test_gpu_matches_reference_goldens(name, ctx, gcz, manifest):
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    if exp["exit"] != 0:
        with pytest.raises(gcz.GczError) as ei:
            _build(ctx, kind, payload, L)
        assert ei.value.code == gcz.GCZ_ERR_SYMBOL
        sym = ei.value.info["error_symbol"]
        sym = sym - 32 if 97 <= sym <= 122 else sym
        assert f"Encountered unknown symbol: {sym} (ASCII code {sym})" == exp["stderr"]
        return
    info = _build(ctx, kind, payload, L)
    assert info["n_strands"] == exp["width"]
    got = gcz.digest(ctx.tree())
    assert compare_digest(got, exp) == {}


@pytest.mark.parametrize("name", ["corpus/chmpxx", "corpus/merged", "fasta/iupac_stress", "lsweep/chmpxx_L16",
                                  "lsweep/chmpxx_L3", "vectors/L16_edges_S5000", "synth/tandem_10000000"])
def test_gpu_wide_table_path(name, ctx_wide, gcz, manifest):
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    _build(ctx_wide, kind, payload, L)
    assert compare_digest(gcz.digest(ctx_wide.tree()), case["expect"]) == {}


@pytest.mark.parametrize("name", ["chmpxx", "hehcmv"])
def test_gpu_full_dump(name, ctx, gcz):
    with open(os.path.join(GOLDEN, "data", name), "rb") as f:
        ctx.build_fasta(f.read(), 12)
    t = ctx.tree()
    with gzip.open(os.path.join(GOLDEN, "full", f"{name}.leaves.bin.gz")) as f:
        assert t.leaves_bin() == f.read()
    with gzip.open(os.path.join(GOLDEN, "full", f"{name}.layers.bin.gz")) as f:
        assert t.layers_bin() == f.read()


def test_gpu_matches_oracle_random_iupac(ctx, gcz, oracle):
    """Random leaves over every nibble value, many sizes (tails, tiny trees)."""
    rng = np.random.default_rng(5)
    for S in [1, 2, 3, 5, 63, 64, 65, 2047, 2048, 2049, 4097, 100_003]:
        pool = rng.integers(0, 1 << 48, size=max(4, S // 7), dtype=np.uint64)
        leaves = pool[rng.integers(0, pool.size, size=S)]
        ctx.build_leaves(leaves, 12)
        g = ctx.tree()
        o = oracle.build_leaves(leaves, 12)
        assert g.leaves_bin() == o.leaves_bin(), S
        assert g.layers_bin() == o.layers_bin(), S
        assert g.root == o.root, S


def test_gpu_deterministic(ctx, gcz):
    data = gcz.synth(1, 3_000_000).tobytes()
    ctx.build_fasta(data, 12)
    a = ctx.tree()
    ctx.build_fasta(data, 12)
    b = ctx.tree()
    assert a.layers_bin() == b.layers_bin() and a.leaves_bin() == b.leaves_bin()


def test_gpu_device_pointer_path(ctx, gcz):
    """gcz_build_device_bases on a device buffer (the bench path), incl. a misaligned pointer."""
    data = gcz.synth(0, 1_000_000)
    ref = gcz.digest((ctx.build_fasta(data.tobytes(), 12), ctx.tree())[1])
    dev = ctx.upload(np.concatenate([np.zeros(1, np.uint8), data]))
    ctx.build_device_bases(dev.ptr + 1, data.size, 12)
    assert compare_digest(gcz.digest(ctx.tree()), ref) == {}
    with pytest.raises(gcz.GczError) as ei:          # aligned path; byte 0 is not a base
        ctx.build_device_bases(dev.ptr, data.size + 1, 12)
    assert ei.value.code == gcz.GCZ_ERR_SYMBOL and ei.value.info["error_offset"] == 0
    leaves = ctx.upload(np.frombuffer(bytes(range(256)) * 8, dtype=np.uint64))
    ctx.build_device_leaves(leaves.ptr, leaves.nbytes // 8, 16)
    dev.free(); leaves.free()


def test_gpu_empty_and_bad_L(ctx, gcz):
    with pytest.raises(gcz.GczError) as ei:
        ctx.build_fasta(b"ACGTACGTAC", 12)
    assert ei.value.code == gcz.GCZ_ERR_EMPTY
    with pytest.raises(gcz.GczError) as ei:
        ctx.build_fasta(b"ACGT" * 100, 17)
    assert ei.value.code == gcz.GCZ_ERR_ARG


@pytest.mark.slow
@pytest.mark.parametrize("name", ["synth/uniform_100000003", "synth/tandem_100000000",
                                  "synth/uniform_1000000000", "synth/tandem_3200000000"])
def test_gpu_large_synth_goldens(name, ctx, gcz, manifest):
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    info = _build(ctx, kind, payload, L)
    exp = case["expect"]
    assert info["n_leaves"] == exp["n_leaves"]
    assert info["layer_size"] == exp["layer_sizes"]
    assert compare_digest(gcz.digest(ctx.tree()), exp) == {}


@pytest.mark.parametrize("env", [{"GCZ_DIRECT": "0"}, {"GCZ_TAIL": "0"}, {"GCZ_DIRECT": "0", "GCZ_TAIL": "0"},
                                 {"GCZ_NODE_CAP_SHIFT": "0"}, {"GCZ_LEAF_CAP_LOG2": "20"},
                                 {"GCZ_PREDUP": "1"}, {"GCZ_PREDUP": "2"}, {"GCZ_PREDUP": "1", "GCZ_TABLE": "wide"},
                                 {"GCZ_BUCKET": "0"}, {"GCZ_BUCKET_MIN": "1"},
                                 {"GCZ_BUCKET_MIN": "1", "GCZ_DIRECT": "0"},
                                 {"GCZ_BUCKET_MIN": "1", "GCZ_PREDUP": "2"}, {"GCZ_FUSED": "0"},
                                 {"GCZ_FUSED": "0", "GCZ_GRAPH": "0"}, {"GCZ_GRAPH": "0", "GCZ_TAIL": "0"},
                                 {"GCZ_DEDUPE_BM": "0"}, {"GCZ_DEDUPE_BM": "0", "GCZ_BUCKET_MIN": "1"},
                                 {"GCZ_DENSE_NB": "1024"}, {"GCZ_DENSE_NB": "1024", "GCZ_DENSE": "2"},
                                 {"GCZ_DENSE": "2", "GCZ_DL_XCD": "0"}, {"GCZ_DENSE": "2", "GCZ_DL_XCD": "15"},
                                 {"GCZ_DENSE": "2", "GCZ_DL_FBW": "0"}, {"GCZ_PART_WORDS": "1", "GCZ_BUCKET_MIN": "1"},
                                 {"GCZ_BUCKET_MIN": "1", "GCZ_PREDUP": "2", "GCZ_DEDUPE_BM": "0"},
                                 {"GCZ_BUCKET_MIN": "1", "GCZ_BKT_XCD": "0"}])
def test_gpu_schedule_knobs_same_tree(env, gcz, manifest):
    """The per-level fallbacks (no direct subtrees, no fused top, tight tables, a leaf
    table that overflows and regrows) build the same tree as the default schedule."""
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = gcz.Context(0)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        for name in ("synth/uniform_10000000", "synth/tandem_10000000", "corpus/merged"):
            case = manifest[name]
            kind, payload, L = case_input(case, gcz)
            _build(c, kind, payload, L)
            assert compare_digest(gcz.digest(c.tree()), case["expect"]) == {}, (env, name)
    finally:
        c.close()


def test_gpu_bucketed_matches_oracle_random(ctx_bucket, gcz, oracle):
    """Bucketed insert on random leaf mixes (unique-heavy and repeat-heavy), against the oracle."""
    rng = np.random.default_rng(11)
    for S, pool_div in [(5, 1), (4097, 1), (100_003, 1), (100_003, 7), (300_001, 50_000)]:
        pool = rng.integers(0, 1 << 48, size=max(4, S // pool_div), dtype=np.uint64)
        leaves = pool[rng.integers(0, pool.size, size=S)]
        ctx_bucket.build_leaves(leaves, 12)
        g = ctx_bucket.tree()
        o = oracle.build_leaves(leaves, 12)
        assert g.leaves_bin() == o.leaves_bin(), S
        assert g.layers_bin() == o.layers_bin(), S


def test_gpu_bucket_overflow_rebuilds(gcz, oracle):
    """Hot keys (more records than a bucket's LDS table holds) with the repeat probe off:
    the bucketed insert overflows and the build reruns on the table -- same tree."""
    saved = {k: os.environ.get(k) for k in ("GCZ_BUCKET_MIN", "GCZ_PREDUP")}
    os.environ.update({"GCZ_BUCKET_MIN": "1", "GCZ_PREDUP": "2"})
    try:
        c = gcz.Context(0)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        rng = np.random.default_rng(12)
        pool = rng.integers(0, 1 << 48, size=3, dtype=np.uint64)
        hot = pool[rng.integers(0, 3, size=200_000)]          # 9 pair keys, ~11 K records each
        cold = rng.integers(0, 1 << 48, size=50_001, dtype=np.uint64)
        leaves = np.concatenate([hot, cold])
        info = c.build_leaves(leaves, 12)
        o = oracle.build_leaves(leaves, 12)
        assert c.tree().leaves_bin() == o.leaves_bin()
        assert c.tree().layers_bin() == o.layers_bin()
        assert info["bucketed_pairs"] == 0   # the final (table) build bucketed nothing
    finally:
        c.close()


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


@pytest.mark.parametrize("env", [{}, {"GCZ_TABLE": "wide"}, {"GCZ_PREDUP": "1"}, {"GCZ_TAIL": "0"},
                                 {"GCZ_PREDUP": "1", "GCZ_TABLE": "wide", "GCZ_TAIL": "0"}, {"GCZ_FUSED": "0"}])
def test_gpu_fused_small_levels_random(env, gcz, oracle):
    """Small builds run two launches per node level (the insert settles the previous
    level's repeats, tables in rotating regions): random leaf mixes from all-unique to
    nearly all-repeated, each built three times (eager, graph capture, graph replay),
    against the oracle."""
    c = _ctx_env(gcz, env)
    rng = np.random.default_rng(23)
    try:
        for S, pool_div in [(3, 1), (257, 1), (2049, 3), (4099, 3), (20_001, 40), (100_003, 1), (100_003, 7),
                            (131_071, 1000), (131_072, 50_000)]:
            pool = rng.integers(0, 1 << 48, size=max(4, S // pool_div), dtype=np.uint64)
            leaves = pool[rng.integers(0, pool.size, size=S)]
            o = oracle.build_leaves(leaves, 12)
            for rep in range(3):
                c.build_leaves(leaves, 12)
                g = c.tree()
                assert g.leaves_bin() == o.leaves_bin(), (env, S, pool_div, rep)
                assert g.layers_bin() == o.layers_bin(), (env, S, pool_div, rep)
    finally:
        c.close()


def test_gpu_repetitive_decision_after_failed_dense_pack(gcz):
    """a genome the dense pack rejects (one IUPAC 'N', past the probe's sample) falls
    back to the hash-table leaf level, whose own repetitive-data probe must decide alone -- the
    dense probe's counts over the rejected pre-words are cleared.  With 3.5 % in-block repeats
    (below the 5 % threshold) both probes together would read 7 % and flip the decision; the
    verdict (gcz_info.repetitive) and the tree must equal those of a build that never tries the
    dense level."""
    rng = np.random.default_rng(5)
    L, S = 12, 1 << 22
    strands = rng.integers(0, 4, size=(S, L), dtype=np.uint8)
    blocks = strands.reshape(S // 256, 256, L)
    for j in range(9):                                   # 9 of 256 strands repeat one earlier in the block
        blocks[:, 200 + j] = blocks[:, 10 + j]
    bases = np.frombuffer(b"ACGT", np.uint8)[strands].tobytes()
    data = b">x\n" + bases[:-1] + b"N\n"               # the last strand: not pure ACGT (N is valid IUPAC)
    got = {}
    for env in ({}, {"GCZ_DENSE": "0"}):
        c = _ctx_env(gcz, env)
        try:
            info = c.build_fasta(data, L)
            assert info["status"] == 0
            got[bool(env)] = (info["repetitive"], info["leaf_path"], gcz.digest(c.tree())["sha_dag"])
        finally:
            c.close()
    assert got[False][1] == got[True][1] == 0, got       # both took the hash-table leaf level
    assert got[False][0] == got[True][0] == 0, got
    assert got[False][2] == got[True][2], got


@pytest.fixture(scope="module")
def ctx_dense_bucket(gcz):
    """Dense leaf level at every size and the two-pass bucketed insert on every hashed level:
    on data the dense probe finds non-repetitive, layer 0 and up take the bitmap-filtered dedupe
    (k_bkt_dedupe_bm); GCZ_PREDUP=2 keeps the block collapse off whatever the probe says."""
    os.environ.update({"GCZ_DENSE": "2", "GCZ_BUCKET_MIN": "1", "GCZ_PREDUP": "2"})
    try:
        c = gcz.Context(0)
    finally:
        for k in ("GCZ_DENSE", "GCZ_BUCKET_MIN", "GCZ_PREDUP"):
            del os.environ[k]
    yield c
    c.close()


@pytest.mark.parametrize("name", [n for n in _names(12_000_000) if not n.startswith("fasta/")])
def test_gpu_bitmap_dedupe_goldens(name, ctx_dense_bucket, gcz, manifest):
    """Every golden through the dense level + bitmap dedupe (or, for IUPAC / L > 12, the table
    levels): the reference's tree bit for bit."""
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    if exp["exit"] != 0:
        return
    _build(ctx_dense_bucket, kind, payload, L)
    assert compare_digest(gcz.digest(ctx_dense_bucket.tree()), exp) == {}


@pytest.mark.parametrize("dups", [0, 200, 20_000, 400_000, 700_000, "hot"])
def test_gpu_bitmap_dedupe_repeats_oracle(dups, ctx_dense_bucket, gcz, oracle):
    """Random ACGT leaves with `dups` copied layer-0 pairs spread over the genome (true repeats
    the bitmaps must route to the exact table: first occurrence, multi, not-first ids) -- up to
    ~700 repeated keys a bucket (700 K) and one pair copied 4000 times (a bucket over the kernel's
    record capacity: handed to k_bkt_dedupe2 in the same build, no rebuild; 6000 copies overflow
    a fine-pass slice, which rebuilds with the table as before).  Equal to the C oracle."""
    rng = np.random.default_rng(900 + (dups if dups != "hot" else 1))
    L, S = 12, 2_400_002
    acgt = np.array([1, 2, 4, 8], dtype=np.uint64)
    codes = rng.integers(0, 4, size=(S, L))
    leaves = (acgt[codes] << (4 * np.arange(L, dtype=np.uint64))).sum(axis=1).astype(np.uint64)
    if dups == "hot":
        dst = rng.choice(S // 2, size=4000, replace=False)
        leaves[2 * dst] = leaves[0]
        leaves[2 * dst + 1] = leaves[1]
    elif dups:
        src = rng.integers(0, S // 2, size=dups)
        dst = rng.integers(0, S // 2, size=dups)
        leaves[2 * dst] = leaves[2 * src]
        leaves[2 * dst + 1] = leaves[2 * src + 1]
    info = ctx_dense_bucket.build_leaves(leaves, L)
    if dups == "hot":   # (the bitmap kernel hands the hot key's bucket back; no rebuild)
        assert info["handed_back"] > 0 and info["attempts"] == 1, info
    g = ctx_dense_bucket.tree()
    o = oracle.build_leaves(leaves, L)
    assert g.leaves_bin() == o.leaves_bin(), dups
    assert g.layers_bin() == o.layers_bin(), dups
    assert g.root == o.root, dups
