"""bench.py's distributed parity check as a world-size-2/3 gloo job on the CPU.

At N > 1 the bench never assembles the tree: every rank streams its slices of
each layer (rank r holds a contiguous id range of every layer) to
rank 0, which hashes them in the ref_harness dump format (leaves.bin, layers.bin).
Here a stand-in group holds rank slices of a tree built by the oracle; the
streamed hashes must equal the hashes of the whole dump -- the format the
reference goldens are stored in (tests/golden/manifest.json).
"""
import hashlib
import json
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


def test_exchange_budget_script_on_committed_probe():
    """scripts/budget.py (DESIGN.md §7's projection) reads a committed virtual-rank line and
    prints, per assumed link bandwidth, T_R = kernels + transfers + collective latency; the
    printed sum and speed-up follow from the line's own numbers."""
    import re
    import subprocess
    import sys
    line = os.path.join(REPO, "profiles", "r04", "strong_virtual8.json")
    out = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "budget.py"), line, "2.5"],
                         capture_output=True, text=True, check=True).stdout
    with open(line) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    rows = re.findall(r"B = ([\d.]+) GB/s: kernels ([\d.]+) \+ transfers ([\d.]+) \+ (\d+) collectives / (\d+) syncs "
                      r"([\d.]+) = ([\d.]+) ms -> ([\d.]+)x", out)
    assert len(rows) == 2
    assert float(rows[0][1]) == round(max(d["rank_kernel_ms"]), 3)
    assert int(rows[0][3]) == len(d["rank_timeline"][0]["exchange_log"])
    for _, k, x, _, _, lat, tot, sp in rows:
        assert abs(float(k) + float(x) + float(lat) - float(tot)) < 2e-3
        assert abs(2.5 / float(tot) - float(sp)) < 0.01


def test_exchange_budget_overlap_model_on_r05_probes():
    """The overlap model (scripts/budget.py, the fused schedule's dependencies replayed) on the
    committed r05 probes: a projection never below the slowest rank's summed segments plus the
    schedule's latencies, never above the additive model's, and faster links never slower; the
    K2 bulk transfer starts at or after R1a's read."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("budget", os.path.join(REPO, "scripts", "budget.py"))
    budget = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(budget)
    for name in ("strong_virtual8.json", "strong_virtual4.json", "strong_virtual2.json", "weak_virtual8_uniform_8g.json"):
        with open(os.path.join(REPO, "profiles", "r05", name)) as f:
            d = json.loads(f.read().strip().splitlines()[-1])
        tl = d["rank_timeline"]
        R = len(tl)
        logs = [r["exchange_log"] for r in tl]
        names = [e[1] for e in logs[0]]
        xb = budget.busiest_bytes(logs, R)
        segs = [r["segments_ms"] for r in tl]
        assert all(len(s) == 9 for s in segs), name
        lat = (len(names) * budget.LAT_US + 2 * budget.SYNC_US) * 1e-3
        floor = max(sum(s) for s in segs) + lat - budget.LAT_US * 1e-3   # (K2's latency overlaps)
        prev = None
        for B in (25.0, 50.0, 100.0):
            T, ev = budget.overlap_model(segs, names, xb, B * 1e9)
            T *= 1e3
            additive = max(d["rank_kernel_ms"]) + sum(xb) / (B * 1e9) * 1e3 + lat
            assert floor - 1e-6 <= T <= additive + 1e-6, (name, B, floor, T, additive)
            if prev is not None:
                assert T <= prev + 1e-9, (name, B)
            prev = T
            ends = {f: (t0, t1) for f, t0, t1 in ev}
            assert ends["K2 (bulk)"][0] >= ends["R1a"][1] - 1e-12, name


def _committed_lines(min_round=5):
    """(path, line) of every committed bench line under profiles/r05 and later (rounds 1-4 used
    a per-build byte model that charged distributed ranks for the whole genome's pairs)."""
    import glob
    import re
    out = []
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r0*", "**", "*.json"), recursive=True)):
        m = re.search(r"profiles/r(\d+)", path)
        if not m or int(m.group(1)) < min_round:
            continue
        with open(path) as f:
            for ln in f.read().splitlines():
                if ln.startswith("{") and '"kernels"' in ln:
                    out.append((path, json.loads(ln)))
    return out


def test_committed_profiles_stay_below_peak():
    """no kernel of a committed bench line is credited above the 8 TB/s HBM peak,
    and the line's roofline names a kernel that moves bytes, with frac <= 1."""
    for path, d in _committed_lines():
        for name, k in d["kernels"].items():
            assert k["gbs"] is None or k["gbs"] <= 8000.0, (path, name, k["gbs"])
        rf = d["roofline"]
        assert rf["alg_bytes_per_launch"] > 0, path
        assert 0.0 < rf["frac"] <= 1.0, (path, rf["frac"])


def test_rank_byte_model_on_the_r04_probes():
    """The per-rank byte model (bench.dist_rank_bytes) over the r04 virtual-rank probes' own
    kernel times: every kernel of rank 0 stays below the HBM peak (the r04 lines credited
    node_insert with 23.9 / 44.4 TB/s by charging a rank for every pair of the genome)."""
    bench = _load_bench()
    for name, S, R in (("strong_virtual8.json", 83_333_333, 8), ("weak_virtual8_uniform_8g.json", 666_666_666, 8),
                       ("strong_virtual2.json", 83_333_333, 2)):
        with open(os.path.join(REPO, "profiles", "r04", name)) as f:
            d = json.loads(f.read().strip().splitlines()[-1])
        # rank 0's strands as the r04 partition gave them: 700 / 850 permille shares
        g = 1 << 9
        T = (S + R - 1) // R
        B = (T + g - 1) // g * g
        Sr = max(g, B * (700 if R >= 5 else 850) // 1000 // g * g)
        c0 = int(d["build"]["n_leaves"] * 0.9)
        for kname, k in d["kernels"].items():
            b = bench.dist_rank_bytes(kname, 12, Sr, 0, R, c0, (Sr + 1) // 2, d["build"]["n_leaves"])
            if b and k["total_ms"] > 0:
                assert b / (k["total_ms"] * 1e-3) / 1e9 <= 8000.0, (name, kname)


def test_bench_reads_the_newest_traffic_capture():
    """The bench line's counter bytes come from the newest round's PMC capture of its config
    (profiles/rNN/pmc_traffic_<config>.json, written by scripts/traffic_json.py from the round's
    final evidence run); no stale copy elsewhere can shadow it, and the capture's total is the
    sum of its kernels."""
    import glob
    import re
    bench = _load_bench()
    assert not glob.glob(os.path.join(REPO, "profiles", "traffic_*.json"))
    for cfg in ("uniform_1g", "tandem_3g2"):
        files = glob.glob(os.path.join(REPO, "profiles", "r*", f"pmc_traffic_{cfg}.json"))
        newest = max(files, key=lambda p: int(re.search(r"[/\\]r(\d+)[/\\]", p).group(1)))
        assert bench.traffic_file(cfg) == newest
        with open(newest) as f:
            tj = json.load(f)
        assert tj["build_total"] == sum(tj["per_build"].values())
        assert tj["config"] == cfg
