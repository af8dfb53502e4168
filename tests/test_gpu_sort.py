"""Frequency sort, bytes() and the .dag writer on the device
against the reference goldens (sorted .dag sha256 = `compress` output) and the host
restatement of sort_tree (src/shared_tree.cpp:443-513)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_input

pytestmark = pytest.mark.gpu


def _names(max_bases):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        m = json.load(f)
    return [n for n, c in sorted(m.items())
            if c["expect"]["exit"] == 0 and not (c["kind"] == "synth" and c["nbases"] > max_bases)
            and c["kind"] != "fastabig" and "buffer" not in c]


@pytest.fixture(scope="module")
def ctx(gcz):
    c = gcz.Context(0)
    yield c
    c.close()


def _build(ctx, kind, payload, L):
    return ctx.build_fasta(payload, L) if kind == "fasta" else ctx.build_leaves(payload, L)


@pytest.mark.parametrize("name", _names(12_000_000))
def test_device_sort_and_dag_match_reference(name, ctx, gcz, manifest):
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    _build(ctx, kind, payload, L)
    host = ctx.tree()                      # unsorted, sorted below on the host
    assert ctx.bytes_device() == exp["unsorted_bytes"]
    ctx.sort_device()
    assert ctx.bytes_device() == exp["bytes"]
    dag = ctx.serialize_device()
    assert len(dag) == exp["bytes"]
    assert hashlib.sha256(dag).hexdigest() == exp["sha_dag"]
    dev = ctx.tree()
    host.sort()
    assert np.array_equal(dev.leaves(), host.leaves())
    for k in range(host.n_layers):
        assert np.array_equal(dev.layer(k), host.layer(k)), k
    assert dev.root == host.root


@pytest.mark.parametrize("name", ["corpus/merged", "synth/uniform_10000000"])
def test_device_sort_after_reserve(name, gcz, manifest):
    """gcz_sort_reserve (the drop-in calls it on a side thread during the fetch) then the sort
    in a fresh context: same .dag as the reference; reserving twice is a no-op."""
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    c = gcz.Context(0)
    try:
        _build(c, kind, payload, L)
        assert gcz._lib.gcz_sort_reserve(c._h) == 0
        assert gcz._lib.gcz_sort_reserve(c._h) == 0
        c.sort_device()
        assert hashlib.sha256(c.serialize_device()).hexdigest() == case["expect"]["sha_dag"]
    finally:
        c.close()


def test_device_sort_idempotent_and_unsorted_dag(ctx, gcz, manifest):
    case = manifest["corpus/hehcmv"]
    kind, payload, L = case_input(case, gcz)
    _build(ctx, kind, payload, L)
    assert hashlib.sha256(ctx.serialize_device()).hexdigest() == case["expect"]["sha_unsorted_dag"]
    ctx.sort_device()
    first = ctx.serialize_device()
    ctx.sort_device()                      # stable sort of sorted counts: identity
    assert ctx.serialize_device() == first


@pytest.mark.slow
@pytest.mark.parametrize("name", ["synth/uniform_1000000000", "synth/tandem_3200000000"])
def test_device_sort_large(name, ctx, gcz, manifest):
    case = manifest[name]
    exp = case["expect"]
    kind, payload, L = case_input(case, gcz)
    buf = ctx.upload(np.frombuffer(payload, dtype=np.uint8))
    ctx.build_device_bases(buf.ptr, len(payload), L)
    buf.free()
    ctx.sort_device()
    dag = ctx.serialize_device()
    assert hashlib.sha256(dag).hexdigest() == exp["sha_dag"]


# ---- decompression: operator[] for every index, on the device ----
SYM = np.frombuffer(b"SACRGBNKTWVDYHM-", dtype=np.uint8)


def _expected_text(kind, payload, L, gcz):
    if kind == "fasta":
        b = np.frombuffer(gcz.fasta_extract(payload, L), dtype=np.uint8)
        b = b[:len(b) // L * L]
        return np.where((b >= 97) & (b <= 122), b - 32, b).astype(np.uint8).tobytes()
    lv = np.asarray(payload, dtype=np.uint64)
    nib = (lv[:, None] >> (4 * np.arange(L, dtype=np.uint64))[None, :]) & np.uint64(15)
    return SYM[nib.astype(np.int64)].tobytes()


@pytest.mark.parametrize("name", _names(12_000_000))
def test_device_decompress_round_trip(name, ctx, gcz, manifest):
    case = manifest[name]
    kind, payload, L = case_input(case, gcz)
    _build(ctx, kind, payload, L)
    expect = _expected_text(kind, payload, L, gcz)
    assert ctx.decompress() == expect
    ctx.sort_device()                      # a permuted tree still spells the same genome
    assert ctx.decompress() == expect


@pytest.mark.slow
def test_device_decompress_1g(ctx, gcz):
    data = gcz.synth(0, 1_000_000_000)
    buf = ctx.upload(data)
    ctx.build_device_bases(buf.ptr, data.size, 12)
    buf.free()
    text = np.frombuffer(ctx.decompress(), dtype=np.uint8)
    up = data[:text.size]
    assert np.array_equal(text, np.where(up >= 97, up - 32, up))
