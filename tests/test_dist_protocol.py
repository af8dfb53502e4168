"""The multi-rank id protocol (csrc/gcz_dist.hip) as a world-size-2/3
gloo job on the CPU.

Each process is one rank: it takes its strand range from the library's own
partition (gcz_dist_plan), dedups locally in first-occurrence order, sends its
keys to their owners (A), gets back first / shared flags (B), ranks its globally
first keys, learns its id offset from an allgather of the counts, and resolves
the other keys through the owner (C / D) -- the same steps the device kernels
take, in numpy over torch.distributed(gloo).  The ids every rank ends with must
be the global first-occurrence ranks of the whole sequence (the reference's
emplace_leaf / emplace_node numbering, src/shared_tree.cpp:630-672), and the
rank-ordered concatenation of the unique keys must be the global unique list.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_gcz


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def owner_of(keys, R):
    h = (keys.astype(np.uint64) * np.uint64(0xFF51AFD7ED558CCD)) & np.uint64((1 << 64) - 1)
    h ^= h >> np.uint64(33)
    return ((h >> np.uint64(32)) * np.uint64(R) >> np.uint64(32)).astype(np.int64)


def first_occurrence_ids(keys):
    """Reference numbering: id = rank of the key's first occurrence."""
    _, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")
    rank_of_class = np.empty_like(order)
    rank_of_class[order] = np.arange(order.size)
    return rank_of_class[inv], keys[np.sort(first)]


def _rank(rank, world, port, keys, out):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    gcz = load_gcz()
    S = keys.size
    s0, s1, _ = gcz.dist_plan(S, world, rank)
    mine = keys[s0:s1]
    # local dedup: local ids in local first-occurrence order
    lid, luniq = first_occurrence_ids(mine) if mine.size else (np.zeros(0, np.int64), mine)
    # A: keys to their owners
    dest = owner_of(luniq, world)
    send = [luniq[dest == d] for d in range(world)]
    sidx = [np.nonzero(dest == d)[0] for d in range(world)]
    got = [None] * world
    dist.all_gather_object(got, send)
    recv = [got[s][rank] for s in range(world)]                      # from each source, in order
    # owner: ranks holding each key
    holders = {}
    for s in range(world):
        for k in recv[s].tolist():
            holders.setdefault(k, []).append(s)
    reply = [np.array([min(holders[k]) != s for k in recv[s].tolist()], dtype=bool) for s in range(world)]
    shared = [np.array([len(holders[k]) > 1 for k in recv[s].tolist()], dtype=bool) for s in range(world)]
    # B: flags back to the senders
    back = [None] * world
    dist.all_gather_object(back, (reply, shared))
    notfirst = np.zeros(luniq.size, dtype=bool)
    is_shared = np.zeros(luniq.size, dtype=bool)
    for d in range(world):
        notfirst[sidx[d]] = back[d][0][rank]
        is_shared[sidx[d]] = back[d][1][rank]
    # globally-first keys, ranked in local order; offsets from an allgather of the counts
    gfirst = ~notfirst
    lrank = np.cumsum(gfirst) - gfirst
    counts = [None] * world
    dist.all_gather_object(counts, int(gfirst.sum()))
    off = int(sum(counts[:rank]))
    gid = np.full(luniq.size, -1, dtype=np.int64)
    gid[gfirst] = off + lrank[gfirst]
    # C: first holders of shared keys send their id; D: owners forward it to the other holders
    cvals = [{int(k): int(g) for k, g, f, sh in zip(luniq[sidx[d]], gid[sidx[d]], gfirst[sidx[d]],
                                                    is_shared[sidx[d]]) if f and sh} for d in range(world)]
    allc = [None] * world
    dist.all_gather_object(allc, cvals)
    table = {}
    for s in range(world):
        table.update(allc[s][rank])
    dvals = [[table[k] for k, nf in zip(recv[s].tolist(), reply[s].tolist()) if nf] for s in range(world)]
    alld = [None] * world
    dist.all_gather_object(alld, dvals)
    for d in range(world):
        need = sidx[d][notfirst[sidx[d]]]
        gid[need] = alld[d][rank]
    assert (gid >= 0).all()
    words = gid[lid] if mine.size else gid[:0]
    res = [None] * world
    dist.all_gather_object(res, (words, luniq[gfirst]))
    if rank == 0:
        out.put((np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", ["repeats", "tandem", "tiny"])
def test_dist_protocol_matches_first_occurrence_ids(world, case):
    rng = np.random.default_rng(world * 7 + len(case))
    if case == "repeats":
        keys = rng.integers(0, 5000, size=40_000).astype(np.int64)
    elif case == "tandem":
        unit = rng.integers(0, 1 << 40, size=37)
        keys = np.concatenate([np.tile(unit, 300), rng.integers(0, 1 << 40, size=20_000)]).astype(np.int64)
    else:
        keys = rng.integers(0, 3, size=5).astype(np.int64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, keys, q)) for r in range(world)]
    for p in procs:
        p.start()
    words, uniq = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect_ids, expect_uniq = first_occurrence_ids(keys)
    assert np.array_equal(words, expect_ids)
    assert np.array_equal(uniq, expect_uniq)
