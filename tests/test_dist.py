"""Multi-rank build (gcz_group) against the reference goldens.

The GPU tests run R virtual ranks on one MI355X (gcz_group_create_local): every
kernel of the distributed path (bucketing, owner tables, id scan, compaction,
remap, gather, tail) runs exactly as with one rank per GPU; only the exchange is
a device copy instead of an RCCL send/recv.  The rank-ordered concatenation of
the slices must equal the reference's tree byte for byte.

The CPU tests check the partition (gcz_dist_plan) properties the algorithm
relies on.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_input, compare_digest


@pytest.fixture(autouse=True)
def deep_distribution(request, monkeypatch):
    """Distribute node levels down to 512 elements per rank (GCZ_DIST_TAIL_LOG2=9), so that
    the small inputs here exercise the distributed node levels; the production default
    (a ~2^23-word tail finished by rank 0) is covered by test_dist_default_depth."""
    if "default_depth" not in request.node.name:
        monkeypatch.setenv("GCZ_DIST_TAIL_LOG2", "9")


# ---- partition (host logic, no GPU) ----------------------------------------------
@pytest.mark.parametrize("S", [1, 2, 7, 9, 100, 1023, 4096, 10085, 1 << 20, 83_333_333, 266_666_666])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_dist_plan_partition(gcz, S, world):
    parts = [gcz.dist_plan(S, world, r) for r in range(world)]
    G = parts[0][2]
    assert all(p[2] == G for p in parts)
    # contiguous, rank order = position order, covers [0, S)
    assert parts[0][0] == 0 and parts[-1][1] == S
    for a, b in zip(parts, parts[1:]):
        assert a[1] == b[0]
    # every nonempty rank boundary is a multiple of 2^G: levels < G pair within a rank
    for s0, s1, _ in parts:
        if s0 < S:
            assert s0 % (1 << G) == 0
    # after G levels each nonempty rank still holds >= 256 elements (except tiny inputs)
    if G > 0:
        sizes = [s1 - s0 for s0, s1, _ in parts if s1 > s0]
        assert min(sizes[:-1] or sizes) >> G >= 256


# ---- GPU: virtual ranks vs the reference ----------------------------------------------
def _cases(max_bases, kinds=("fasta", "synth", "leaves")):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        m = json.load(f)
    out = []
    for n, c in sorted(m.items()):
        if c["kind"] not in kinds or c["expect"]["exit"] != 0 or "buffer" in c:
            continue
        if c["kind"] == "synth" and c["nbases"] > max_bases:
            continue
        out.append(n)
    return out


def _dist_build(gcz, group, kind, payload, L):
    """Upload the whole input once, hand every virtual rank a pointer to its strands."""
    ctx0 = group.ctx(0)
    if kind == "fasta":
        bases = np.frombuffer(gcz.fasta_extract(payload, L), dtype=np.uint8)
        S = len(bases) // L
        buf = ctx0.upload(bases if len(bases) else np.zeros(1, np.uint8))
        ptrs = [buf.ptr + gcz.dist_plan(max(S, 1), group.world, r)[0] * L for r in range(group.world)]
        try:
            return group.build_device_bases(ptrs, S, L)
        finally:
            buf.free()
    leaves = np.ascontiguousarray(payload, dtype=np.uint64)
    S = leaves.size
    buf = ctx0.upload(leaves if S else np.zeros(1, np.uint64))
    ptrs = [buf.ptr + gcz.dist_plan(max(S, 1), group.world, r)[0] * 8 for r in range(group.world)]
    try:
        return group.build_device_leaves(ptrs, S, L)
    finally:
        buf.free()


@pytest.fixture(scope="module")
def groups(gcz):
    gs = {}
    yield lambda w: gs.setdefault(w, gcz.Group.local(w))
    for g in gs.values():
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("name", _cases(12_000_000))
def test_dist_matches_reference_goldens(name, world, gcz, manifest, groups):
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    g = groups(world)
    info = _dist_build(gcz, g, kind, payload, L)
    assert info["n_strands"] == exp["width"]
    got = gcz.digest(g.tree())
    assert compare_digest(got, exp) == {}


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 5, 16])
def test_dist_random_iupac_vs_oracle(world, gcz, oracle, groups):
    """Random IUPAC genomes with planted repeats: every rank holds repeats of the others' keys."""
    rng = np.random.default_rng(7 + world)
    alphabet = np.frombuffer(b"ACGTRYKMBVDHSWN-acgt", dtype=np.uint8)
    for L, n in [(12, 300_000), (5, 77_777), (16, 123_456), (3, 50_001)]:
        base = alphabet[rng.integers(0, 6, size=n)]
        # plant copies of early segments late in the genome (cross-rank repeats)
        for _ in range(20):
            a = int(rng.integers(0, n // 2))
            b = int(rng.integers(n // 2, n - 2000))
            base[b:b + 2000] = base[a:a + 2000]
        data = base.tobytes()
        ref = oracle.build_fasta(data, L)
        info = _dist_build(gcz, groups(world), "fasta", data, L)
        t = groups(world).tree()
        assert info["n_leaves"] == len(ref.leaves())
        assert np.array_equal(t.leaves(), ref.leaves())
        for k in range(ref.n_layers):
            assert np.array_equal(t.layer(k), ref.layer(k)), (L, k)
        assert t.root == ref.root


@pytest.mark.gpu
def test_dist_bad_symbol_reports_first_offset(gcz, groups):
    g = groups(3)
    data = bytearray(gcz.synth(0, 1_200_000).tobytes())
    data[900_001] = ord("x")     # on the last rank
    data[700_005] = ord("!")     # earlier, on rank 1 or 2: this one is reported
    with pytest.raises(gcz.GczError) as ei:
        _dist_build(gcz, g, "fasta", bytes(data), 12)
    assert ei.value.code == gcz.GCZ_ERR_SYMBOL
    assert ei.value.info["error_offset"] == 700_005
    assert ei.value.info["error_symbol"] == ord("!")
    # the group is reusable after an error
    info = _dist_build(gcz, g, "fasta", gcz.synth(0, 100_000).tobytes(), 12)
    assert info["status"] == 0


@pytest.mark.gpu
def test_dist_equals_single_device_tandem(gcz, groups):
    """Tandem repeats (hot keys on every rank): 4 ranks == one device, all layers."""
    data = gcz.synth(1, 20_000_000).tobytes()
    ctx = gcz.Context(0)
    try:
        ctx.build_fasta(data, 12)
        single = ctx.tree()
        _dist_build(gcz, groups(4), "fasta", data, 12)
        multi = groups(4).tree()
        assert np.array_equal(single.leaves(), multi.leaves())
        assert single.n_layers == multi.n_layers
        for k in range(single.n_layers):
            assert np.array_equal(single.layer(k), multi.layer(k)), k
        assert single.root == multi.root
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("world,names", [(2, ("synth/uniform_100000003", "synth/tandem_100000000",
                                              "synth/uniform_1000000000")),
                                         (4, ("synth/uniform_1000000000",)),
                                         (8, ("synth/uniform_100000003", "synth/tandem_100000000",
                                              "synth/uniform_1000000000", "synth/tandem_3200000000"))])
def test_dist_synth_large(world, names, gcz, manifest, groups):
    """The benchmark's genome (1 Gbase uniform: the fused schedule) at 2, 4 and 8 virtual ranks and
    the synthetic goldens around it, against the compiled reference."""
    for name in names:
        case = manifest[name]
        kind, payload, L = case_input(case, gcz)
        _dist_build(gcz, groups(world), kind, payload, L)
        assert compare_digest(gcz.digest(groups(world).tree()), case["expect"]) == {}


@pytest.mark.gpu
def test_dist_rccl_world1(gcz, manifest):
    """The RCCL transport (dlopen'd librccl, communicator, allgather, group calls) with one rank."""
    ctx = gcz.Context(0)
    try:
        g = gcz.Group.rccl(ctx, 0, 1, gcz.dist_unique_id())
        # the bulk communicator (ncclCommSplit), its stream and the two creation agreements ran
        assert g.has_bulk
        for name in ("corpus/chmpxx", "corpus/merged"):
            case = manifest[name]
            kind, payload, L = case_input(case, gcz)
            bases = np.frombuffer(gcz.fasta_extract(payload, L), dtype=np.uint8)
            buf = ctx.upload(bases)
            try:
                g.build_device_bases([buf.ptr], len(bases) // L, L)
            finally:
                buf.free()
            assert compare_digest(gcz.digest(g.tree()), case["expect"]) == {}
        g.close()
    finally:
        ctx.close()


@pytest.mark.gpu
def test_dist_rccl_bulk_kill_switch(gcz, monkeypatch):
    """GCZ_FL_BULK=0: the creation agreement finds a rank that does not want the bulk
    communicator, so no rank splits and bulk groups run in line (the path every test covers)."""
    monkeypatch.setenv("GCZ_FL_BULK", "0")
    ctx = gcz.Context(0)
    try:
        g = gcz.Group.rccl(ctx, 0, 1, gcz.dist_unique_id())
        assert not g.has_bulk
        g.close()
    finally:
        ctx.close()


def _group_with_env(gcz, world, env):
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


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["1", "2", "2w"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_dist_local_dedupe_modes(mode, world, gcz, manifest, oracle):
    """Node levels with (GCZ_DIST_LOCAL=1) and without (=2) the local dedupe: without it a
    key reaches its owner once per occurrence, several times from one rank, and the owner
    takes the first record in receive order (stable bucketing) as the first occurrence --
    through the position-packed owner table, or (2w, GCZ_TABLE=wide) the wide slots."""
    env = {"GCZ_DIST_LOCAL": mode[0]}
    if mode.endswith("w"):
        env["GCZ_TABLE"] = "wide"
    g = _group_with_env(gcz, world, env)
    try:
        for name in ("corpus/chmpxx", "corpus/merged", "synth/uniform_10000000", "synth/tandem_10000000"):
            case = manifest[name]
            kind, payload, L = case_input(case, gcz)
            _dist_build(gcz, g, kind, payload, L)
            assert compare_digest(gcz.digest(g.tree()), case["expect"]) == {}, name
        rng = np.random.default_rng(world)
        alphabet = np.frombuffer(b"ACGTRYKMBVDHSWN-", dtype=np.uint8)
        base = alphabet[rng.integers(0, 4, size=400_000)]
        for _ in range(30):     # repeats inside one rank and across ranks
            a = int(rng.integers(0, 390_000))
            b = int(rng.integers(0, 390_000))
            base[b:b + 5000] = base[a:a + 5000]
        data = base.tobytes()
        ref = oracle.build_fasta(data, 6)
        _dist_build(gcz, g, "fasta", data, 6)
        t = g.tree()
        assert np.array_equal(t.leaves(), ref.leaves())
        for k in range(ref.n_layers):
            assert np.array_equal(t.layer(k), ref.layer(k)), k
        assert t.root == ref.root
    finally:
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,name", [(3, "corpus/merged"), (8, "synth/tandem_100000000"),
                                        (8, "synth/uniform_1000000000"), (2, "synth/uniform_100000003")])
def test_dist_default_depth(world, name, gcz, manifest, groups):
    """The default partition depth: distributed levels stop once ~2^23 words are left in
    total (at R = 8: 2^20 per rank) and rank 0 finishes the top alone."""
    assert "GCZ_DIST_TAIL_LOG2" not in os.environ
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    _dist_build(gcz, groups(world), kind, payload, L)
    assert compare_digest(gcz.digest(groups(world).tree()), case["expect"]) == {}


@pytest.mark.gpu
@pytest.mark.parametrize("seed", ["1", "2", "0"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_dist_leaf_dictionary(seed, world, gcz, manifest, oracle, monkeypatch):
    """Rank 0's leaf dictionary (GCZ_DIST_SEED = its first chunks; 0 = off) on small inputs:
    GCZ_LEAF_CHUNKS_FROM forces the chunked leaf level so rank 0 has chunks to share, and
    ranks > 0 seed their tables (strands of dictionary keys take global ids from the probe)."""
    monkeypatch.setenv("GCZ_LEAF_CHUNKS_FROM", "1024")
    monkeypatch.setenv("GCZ_DIST_SEED", seed)
    g = gcz.Group.local(world)
    try:
        for name in ("corpus/chmpxx", "corpus/merged", "synth/uniform_10000000", "synth/tandem_10000000",
                     "fasta/iupac_stress", "corpus/hehcmv"):
            case = manifest[name]
            kind, payload, L = case_input(case, gcz)
            _dist_build(gcz, g, kind, payload, L)
            assert compare_digest(gcz.digest(g.tree()), case["expect"]) == {}, name
        rng = np.random.default_rng(100 + world)
        alphabet = np.frombuffer(b"ACGTRYKMBVDHSWN-", dtype=np.uint8)
        base = alphabet[rng.integers(0, 16, size=300_000)]
        data = base.tobytes()
        ref = oracle.build_fasta(data, 4)
        _dist_build(gcz, g, "fasta", data, 4)
        t = g.tree()
        assert np.array_equal(t.leaves(), ref.leaves())
        for k in range(ref.n_layers):
            assert np.array_equal(t.layer(k), ref.layer(k)), k
    finally:
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_dist_owner_hot_pair_overflow(world, gcz, oracle):
    """Node levels without the local dedupe (GCZ_DIST_LOCAL=2: the owners partition their
    records in LDS buckets) and one pair planted 30,000 times: its owner's slice overflows,
    the build reruns on the tables -- same tree as the oracle."""
    rng = np.random.default_rng(101 + world)
    S = 2_600_000
    leaves = rng.integers(0, 1 << 48, size=S, dtype=np.uint64)
    a, b = np.uint64(0x123456789AB), np.uint64(0xBA987654321)
    js = rng.choice(np.arange(S // 2 + 2**20, S, 2), size=30_000, replace=False)
    leaves[js] = a
    leaves[js + 1] = b
    ref = oracle.build_leaves(leaves, 12)
    g = _group_with_env(gcz, world, {"GCZ_DIST_LOCAL": "2"})
    try:
        _dist_build(gcz, g, "leaves", leaves, 12)
        t = g.tree()
        assert np.array_equal(t.leaves(), ref.leaves())
        for k in range(ref.n_layers):
            assert np.array_equal(t.layer(k), ref.layer(k)), k
        assert t.root == ref.root
    finally:
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_dist_skewed_repetitive_slice(world, gcz, groups):
    """Repetitive data on the LAST rank only (uniform everywhere else): only that rank's probe
    sees in-block repeats, the OR over the ranks turns the local dedupe on for every rank
    (written back into each rank's header), and the tree equals the single-device build."""
    n = 16_000_000
    uni = gcz.synth(0, n).tobytes()
    tan = gcz.synth(1, n).tobytes()
    cut = n - n // (world * 2)           # inside the last rank's slice
    data = uni[:cut] + tan[cut:]
    ctx = gcz.Context(0)
    try:
        ctx.build_fasta(data, 12)
        single = ctx.tree()
        _dist_build(gcz, groups(world), "fasta", data, 12)
        multi = groups(world).tree()
        assert np.array_equal(single.leaves(), multi.leaves())
        assert single.n_layers == multi.n_layers
        for k in range(single.n_layers):
            assert np.array_equal(single.layer(k), multi.layer(k)), k
        assert single.root == multi.root
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_dist_assemble_device_ratio_path(world, gcz, manifest, groups):
    """A distributed tree gathered device to device into one context (gcz_group_assemble):
    that context's frequency sort and .dag writer give the reference .dag (sort_tree / bytes /
    serialize on the device, no host gather), its decompression gives the genome back, and the
    fetched tree equals the golden dumps."""
    import hashlib
    ctx = gcz.Context(0)
    try:
        for name in ("corpus/chmpxx", "corpus/merged", "synth/uniform_10000000", "synth/tandem_10000000"):
            case = manifest[name]
            exp = case["expect"]
            kind, payload, L = case_input(case, gcz)
            _dist_build(gcz, groups(world), kind, payload, L)
            groups(world).assemble(ctx)
            assert compare_digest(gcz.digest(ctx.tree()), exp) == {}, name
            if kind == "fasta":
                bases = gcz.fasta_extract(payload)
                bases = bases[:len(bases) // L * L].upper()
                assert ctx.decompress() == bases, name
            ctx.sort_device()
            assert hashlib.sha256(ctx.serialize_device()).hexdigest() == exp["sha_dag"], name
    finally:
        ctx.close()
