"""Single-device builds of more than 2^29 - 1 strands.

The single-device build keeps positions in the 29-bit index field of its words; the
reference bounds only ids to 29 bits and builds longer genomes (src/shared_tree.cpp:630-672,
743-763: size_t positions, segments of 2^25 strands).  libgcz builds them as virtual ranks on
the same device whose slices are concatenated into the context's arrays (gcz_split_build,
csrc/gcz_dist.hip).  GCZ_SPLIT_MIN / GCZ_SPLIT_SHARE force that path on small genomes, so
every golden can pin it; the slow tests run the real thing on the compiled reference's
8 Gbase (667 M strands, L = 12) and 600 Mbase at L = 1 (600 M strands) goldens.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, case_input, compare_digest

pytestmark = pytest.mark.gpu


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


@pytest.fixture(scope="module")
def ctx_split(gcz):
    """Every build through the virtual-rank split, 2^15 strands per rank (up to 26 ranks here)."""
    c = _ctx_env(gcz, {"GCZ_SPLIT_MIN": "0", "GCZ_SPLIT_SHARE": "32768"})
    yield c
    c.close()


SPLIT_CASES = ["corpus/chmpxx", "corpus/hehcmv", "corpus/merged", "corpus/humdyst", "corpus/vaccg",
               "lsweep/chmpxx_L1", "lsweep/chmpxx_L5", "lsweep/chmpxx_L13", "lsweep/chmpxx_L16",
               "synth/uniform_1000000", "synth/uniform_10000000", "synth/tandem_10000000"]


@pytest.mark.parametrize("name", SPLIT_CASES)
def test_gpu_split_goldens(name, ctx_split, gcz, manifest):
    """The split build (forced) equals the compiled reference on corpus, IUPAC, L-sweep and
    synthetic goldens, through the host digest and the device ratio path."""
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    info = ctx_split.build_fasta(payload, L) if kind == "fasta" else ctx_split.build_leaves(payload, L)
    exp = case["expect"]
    assert info["n_strands"] == exp["width"]
    assert compare_digest(gcz.digest(ctx_split.tree()), exp) == {}
    # the assembled arrays serve the device sort, .dag writer and decompression
    ctx_split.sort_device()
    assert hashlib.sha256(ctx_split.serialize_device()).hexdigest() == exp["sha_dag"]


def test_gpu_split_roundtrip_and_leaves(ctx_split, gcz, oracle):
    """Leaf input (shared_tree(std::vector<dna>&)) through the split against the oracle, and
    the decompression round trip of a split FASTA build."""
    rng = np.random.default_rng(31)
    for S, pool_div in [(40_001, 1), (100_003, 9), (70_000, 20_000)]:
        pool = rng.integers(0, 1 << 48, size=max(4, S // pool_div), dtype=np.uint64)
        leaves = pool[rng.integers(0, pool.size, size=S)]
        ctx_split.build_leaves(leaves, 12)
        g = ctx_split.tree()
        o = oracle.build_leaves(leaves, 12)
        assert g.leaves_bin() == o.leaves_bin(), S
        assert g.layers_bin() == o.layers_bin(), S
        assert g.root == o.root
    data = gcz.synth(1, 2_000_003).tobytes()
    info = ctx_split.build_fasta(data, 12)
    assert info["n_strands"] == len(data) // 12
    assert ctx_split.decompress() == data[: len(data) // 12 * 12].upper()


def test_gpu_split_errors(ctx_split, gcz, manifest):
    """An unknown symbol is reported at the same byte offset through the split."""
    exp = manifest["fasta/bad_symbol"]["expect"]
    assert exp["exit"] == 1
    with open(os.path.join(GOLDEN, "fasta", "bad_symbol.fa"), "rb") as f:
        data = f.read()
    with pytest.raises(gcz.GczError) as ei:
        ctx_split.build_fasta(data, 12)
    assert ei.value.code == gcz.GCZ_ERR_SYMBOL
    ref = gcz.Context(0)
    try:
        with pytest.raises(gcz.GczError) as e2:
            ref.build_fasta(data, 12)
        assert (ei.value.info["error_offset"], ei.value.info["error_symbol"]) == \
               (e2.value.info["error_offset"], e2.value.info["error_symbol"])
    finally:
        ref.close()


def _device_digest(ctx, gcz, nbases, L, kind):
    """Build `nbases` synthetic bases resident in HBM; hashes of the raw dump (leaves,
    layers), the unsorted and the sorted .dag, all written or sorted on the device."""
    host = gcz.synth(kind, nbases)
    buf = ctx.upload(host)
    del host
    try:
        info = ctx.build_device_bases(buf.ptr, nbases, L)
    finally:
        buf.free()
    d = {"n_leaves": info["n_leaves"], "layer_sizes": info["layer_size"], "root": info["root"],
         "width": info["n_strands"], "depth": info["n_layers"] + 1,
         "sha_unsorted_dag": hashlib.sha256(ctx.serialize_device()).hexdigest()}
    t = ctx.tree()
    d["sha_leaves_bin"] = hashlib.sha256(t.leaves_bin()).hexdigest()
    h = hashlib.sha256()
    for k in range(t.n_layers):
        w = t.layer(k)
        h.update(np.uint64(len(w) // 2).astype("<u8").tobytes())
        h.update(w.astype("<u4").tobytes())
    d["sha_layers_bin"] = h.hexdigest()
    del t
    ctx.sort_device()
    d["bytes"] = ctx.bytes_device()
    d["sha_dag"] = hashlib.sha256(ctx.serialize_device()).hexdigest()
    return info, d


@pytest.mark.slow
@pytest.mark.parametrize("name", ["synth/uniform_8000000000", "synth/uniform_600000000_L1"])
def test_gpu_split_beyond_2p29_strands(name, gcz, manifest):
    """More than 2^29 - 1 strands on ONE device (no GCZ_SPLIT_* knobs): the compiled
    reference's 8 Gbase golden (L = 12, 666,666,666 strands) and 600 Mbase at L = 1."""
    if name not in manifest:
        pytest.skip(f"{name} golden not generated")
    case = manifest[name]
    exp = case["expect"]
    assert exp["width"] > (1 << 29) - 1
    ctx = gcz.Context(0)
    try:
        info, got = _device_digest(ctx, gcz, case["nbases"], case["L"], case["synth_kind"])
    finally:
        ctx.close()
    assert info["status"] == 0
    diffs = {k: (v, exp.get(k)) for k, v in got.items() if v != exp.get(k)}
    assert diffs == {}


@pytest.mark.slow
def test_compress_cli_beyond_2p29_strands(gcz, manifest, tmp_path):
    """The drop-in CLI (shared_tree{path}) no longer exits on > 2^29 - 1 strands:
    compress --dna-size=1 on the 600 Mbase genome writes the reference's .dag."""
    name = "synth/uniform_600000000_L1"
    if name not in manifest:
        pytest.skip(f"{name} golden not generated")
    case = manifest[name]
    exp = case["expect"]
    src = tmp_path / "g600m.txt"
    gcz.synth(case["synth_kind"], case["nbases"]).tofile(str(src))
    out = tmp_path / "g600m.dag"
    r = subprocess.run([os.path.join(PKG, "compress"), "--statistics", "--dna-size=1", f"--output={out}", str(src)],
                       capture_output=True, text=True, cwd=str(tmp_path), timeout=600)
    assert r.returncode == 0, r.stderr
    f = r.stdout.strip().splitlines()[-1].split(",")   # (the CLI echoes the --dna-size value first)
    assert f[0] == "1" and int(f[1]) == exp["width"] and f[2] == exp["ratio"] and int(f[4]) == exp["bytes"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == exp["sha_dag"]
