"""bench.py's distributed parity check as a world-size-2/3 gloo job on the CPU.

At N > 1 the bench never assembles the tree: every rank streams its slices of
each layer (rank r holds a contiguous id range of every layer) to
rank 0, which hashes them in the ref_harness dump format (leaves.bin, layers.bin).
Here a stand-in group holds rank slices of a tree built by the oracle; the
streamed hashes must equal the hashes of the whole dump -- the format the
reference goldens are stored in (tests/golden/manifest.json).
"""
import hashlib
import importlib.util
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, REPO, load_oracle


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _load_bench():
    spec = importlib.util.spec_from_file_location("gcz_bench", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class SliceGroup:
    """Rank `r` of `world` (or `n_local` virtual ranks) holding contiguous slices."""

    def __init__(self, leaves, layers, world, ranks):
        self.leaves, self.layers, self.world, self.ranks = leaves, layers, world, ranks
        self.n_local = len(ranks)

    def _cut(self, n, r):
        b = np.linspace(0, n, self.world + 1).astype(np.int64)
        b[1:-1] = np.minimum(b[1:-1] + np.arange(1, self.world) % 2, n)   # ragged cuts
        return b[r], b[r + 1]

    def copy_slice(self, i, layer):
        r = self.ranks[i]
        if layer < 0:
            a, b = self._cut(self.leaves.size, r)
            return self.leaves[a:b].copy()
        w = self.layers[layer]
        n = w.size // 2
        if n < 4 * self.world:                     # top layers live on rank 0 only
            return w.copy() if r == 0 else w[:0].copy()
        a, b = self._cut(n, r)
        return w[2 * a:2 * b].copy()


def _expected(tree):
    return (hashlib.sha256(tree.leaves_bin()).hexdigest(), hashlib.sha256(tree.layers_bin()).hexdigest())


def _tree():
    oracle = load_oracle()
    with open(os.path.join(GOLDEN, "data", "chmpxx"), "rb") as f:
        return oracle.build_fasta(f.read(), 12)


def _arrays(tree):
    return (np.asarray(tree.leaves(), dtype=np.uint64),
            [np.asarray(tree.layer(k), dtype=np.uint32) for k in range(tree.n_layers)])


def _rank(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    bench = _load_bench()
    tree = _tree()
    leaves, layers = _arrays(tree)
    info = {"n_layers": tree.n_layers, "layer_size": [w.size // 2 for w in layers]}
    d = bench.stream_digest(SliceGroup(leaves, layers, world, [rank]), dist, rank, world, info)
    if rank == 0:
        q.put((d["sha_leaves_bin"], d["sha_layers_bin"]) == _expected(tree))
    dist.destroy_process_group()


def _run(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return ok


def test_stream_digest_world2():
    assert _run(2)


def test_stream_digest_world3():
    assert _run(3)


def test_stream_digest_virtual_ranks():
    """--virtual R: one process holds every rank's slices."""
    bench = _load_bench()
    tree = _tree()
    leaves, layers = _arrays(tree)
    info = {"n_layers": tree.n_layers, "layer_size": [w.size // 2 for w in layers]}
    d = bench.stream_digest(SliceGroup(leaves, layers, 4, [0, 1, 2, 3]), None, 0, 1, info)
    assert (d["sha_leaves_bin"], d["sha_layers_bin"]) == _expected(tree)
