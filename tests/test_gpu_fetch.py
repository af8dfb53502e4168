"""The host fetch of a built DAG (gcz_fetch_host: pinned staging ring + parallel host copies,
the drop-in's path into the shared_tree containers) returns exactly the words the plain
per-layer copies (gcz_copy_leaves / gcz_copy_layer) return: small DAGs (one staging batch)
and DAGs of several ring passes (> 16 MB)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(gcz):
    c = gcz.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("nbases", [1_200, 1_000_000, 60_000_000, 200_000_000])
def test_fetch_host_matches_layer_copies(nbases, ctx, gcz):
    host = gcz.synth(0, nbases)
    dev = ctx.upload(host)
    ctx.build_device_bases(dev.ptr, nbases, 12)
    dev.free()
    info = ctx.info()
    n_leaves, layers = info["n_leaves"], info["layer_size"][: info["n_layers"]]
    lib = gcz._lib
    ref_leaves = np.empty(max(n_leaves, 1), np.uint64)
    assert lib.gcz_copy_leaves(ctx._h, ref_leaves.ctypes.data) == 0
    ref = []
    for k, n in enumerate(layers):
        a = np.empty(max(2 * n, 1), np.uint32)
        assert lib.gcz_copy_layer(ctx._h, k, a.ctypes.data) == 0
        ref.append(a[: 2 * n])
    got_leaves = np.full(max(n_leaves, 1), 7, np.uint64)
    got = [np.full(max(2 * n, 1), 7, np.uint32) for n in layers]
    ptrs = (ctypes.c_void_p * len(got))(*[g.ctypes.data for g in got])
    for _ in range(2):   # a second fetch reuses the staging ring
        assert lib.gcz_fetch_host(ctx._h, got_leaves.ctypes.data, ptrs) == 0
        assert np.array_equal(got_leaves[:n_leaves], ref_leaves[:n_leaves])
        for k, n in enumerate(layers):
            assert np.array_equal(got[k][: 2 * n], ref[k]), k
