#!/usr/bin/env python3
"""Benchmark: shared_tree build throughput (bases/s) on MI355X.

One step = one full device build (leaf pack -> every level's hash-cons ->
unique nodes/leaves + root resident in HBM) of the configured synthetic genome,
with the ASCII bases already resident in HBM (SURVEY §8(d) timing scope).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config uniform_1g]

N > 1 is launched by torch.distributed.run (one process per GPU).  Default
(--mode strong, BASELINE's metric): the configured genome itself (uniform_1g:
1 Gbase) is partitioned over the ranks (gcz_dist_plan: contiguous strand ranges,
rank order = position order); each rank generates only its own bases, and every
hash-consed level reconciles keys through their owner rank with RCCL over xGMI
(gcz_group).  Total work is fixed: "scaling": "strong".  The same
run times the weak-scaled case as an extra field (one genome of N x the config
size, 1 config genome per GPU; --no-weak skips it).  --mode weak makes that the
headline; --mode replicas runs N independent builds of N different genomes (no
data-path collective).  --virtual R (one GPU) runs the distributed path with R
virtual ranks on one device, to measure its per-rank cost.

Printed (rank 0): ONE JSON line with value, roofline of the dominant kernel,
the CPU baseline (compiled reference on this host, the same genome, run beside
the GPU work) and the parity verdict against the reference goldens.  A parity
mismatch exits with status 3 after the line.
"""
import argparse
import hashlib
import importlib.util
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
METRIC = "bases/sec shared_tree build, 1 Gbase synthetic, 1/2/4/8 MI355X; ratio bit-exact"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    "uniform_1g": {"kind": 0, "nbases": 1_000_000_000, "golden": "synth/uniform_1000000000"},
    "uniform_100m": {"kind": 0, "nbases": 100_000_003, "golden": "synth/uniform_100000003"},
    "tandem_100m": {"kind": 1, "nbases": 100_000_000, "golden": "synth/tandem_100000000"},
    "tandem_3g2": {"kind": 1, "nbases": 3_200_000_000, "golden": "synth/tandem_3200000000"},
    # the genomes of the weak-scaled runs (N x uniform_1g), for --virtual probes on one GPU
    "uniform_2g": {"kind": 0, "nbases": 2_000_000_000, "golden": "synth/uniform_2000000000"},
    "uniform_4g": {"kind": 0, "nbases": 4_000_000_000, "golden": "synth/uniform_4000000000"},
    "uniform_8g": {"kind": 0, "nbases": 8_000_000_000, "golden": "synth/uniform_8000000000"},
    # BASELINE configs 2 and 3: the bundled corpus files (FASTA; headers stripped on the host)
    "hehcmv": {"kind": "file", "path": "tests/golden/data/hehcmv", "golden": "corpus/hehcmv"},
    "merged": {"kind": "file", "path": "tests/golden/data/merged", "golden": "corpus/merged"},
}


def genome(gcz, cfg, seed, begin, end):
    """Bases [begin, end) of the configured genome (synthetic, or a corpus file's bases)."""
    if cfg["kind"] == "file":
        with open(os.path.join(REPO, cfg["path"]), "rb") as f:
            b = np.frombuffer(gcz.fasta_extract(f.read()), dtype=np.uint8)
        return b[begin:end].copy()
    out = np.empty(max(end - begin, 1), dtype=np.uint8)
    gcz._lib.gcz_synth_fill(gcz._ptr(out), cfg["kind"], seed, begin, end)
    return out[:end - begin]


def load_gcz():
    path = os.path.join(REPO, "genome-compression_amd", "gcz.py")
    spec = importlib.util.spec_from_file_location("gcz", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["gcz"] = mod
    spec.loader.exec_module(mod)
    return mod


def dense_buckets(C):
    """The dense leaf level's code buckets for a code space of C codes (gcz_ctx::dense_nb = 512,
    at least C / 2^14: a bucket's LDS table holds <= 2^14 codes)."""
    return min(C, max(512, C >> 14))


def algorithmic_bytes(kernel, L, S, n_leaves, layer_sizes, hashed_pairs=None, bucketed_pairs=0, two_pass=False,
                      launches=None, repetitive=False):
    """Algorithmic HBM bytes of all launches of `kernel` in one build:
    streamed bytes + one 64-B sector per random table/group access.  The per-level kernels
    (flagscan_node, resolve_node) count only the levels they ran on: the first `launches`
    node levels (the later ones are direct subtrees or the fused tail)."""
    pk = []
    n = S
    while True:
        p = (n + 1) // 2
        pk.append(p)
        if p == 1:
            break
        n = p
    U = n_leaves
    if kernel == "leaf_insert":     # ASCII in, provisional word out, one table sector per strand
        return S * L + 4 * S + 64 * S
    if kernel == "node_insert":     # pair + child marks in, word out, a table sector: per pair it
        # inserted (the hashed pairs that did not go through the buckets; bucketed levels
        # and direct ones return at the gate)
        hashed = (hashed_pairs if hashed_pairs is not None else sum(pk)) - bucketed_pairs
        if hashed <= 0:             # every hashed level went through the buckets: gate-only launches
            return 0
        return (8 + 4 + 4 + 64) * hashed
    # bucketed node insert (non-repetitive data, levels of >= 2^20 pairs: layer 0 of
    # uniform_1g): bp = hashed pairs that went through the buckets
    bp = bucketed_pairs
    if kernel == "bucket_count":    # pair in (and the per-chunk bucket counts out)
        return 8 * bp + 4 * (bp // 3072 + 1) * ((bp >> 16) + 1)
    if kernel == "bucket_scan":     # exclusive scan of the count matrix
        return 8 * (bp // 3072 + 1) * ((bp >> 16) + 1)
    if two_pass and kernel == "bucket_scatter":   # two-pass partition, pass 1 (k_bkt_part): EVERY pair of
        # the levels it ran on streams through it -- pair (8) and, above layer 0, both children's
        # marks (4) in; with the block collapse (repetitive data) the provisional word (4), and its
        # own two marks (2) out -- and each bucketed pair appends an 8-B record to a coarse run
        # (round 5 charged the records' pairs only, which made the repetitive config's counter bytes
        # look 2.6x the algorithmic ones: the read / write split of profiles/r06 matches this stream)
        lv = pk[:launches] if launches is not None else pk[:1]
        return sum(p * (8 + (4 if k else 0) + (4 if repetitive else 0) + 2) for k, p in enumerate(lv)) + 8 * bp
    if kernel == "bucket_fine":     # pass 2: records in, re-encoded records out (LDS-sorted slices)
        return 16 * bp
    if kernel == "bucket_scatter":  # pair in, word out, one 8-B record store (a 64-B sector) per pair
        return 12 * bp + 64 * bp
    if kernel == "bucket_dedupe":   # records in; repeats: mark + word sectors
        return 8 * bp + 128 * max(0, bp - (layer_sizes[0] if layer_sizes else bp))
    # dense leaf level (pure ACGT, L <= 12; gcz_dense.h): streamed bytes per pass
    nch = (S + 32767) // 32768
    C = 2 ** (2 * L - 1)            # the code space: canonical codes (top bit 0, gcz_dense.h)
    NB = dense_buckets(C)
    if kernel == "dl_pack":         # bases in, pre-word out, per-chunk bucket counts
        return S * L + 4 * S + 4 * NB * nch
    if kernel == "dl_scan":         # exclusive scan of the count matrix
        return 8 * NB * nch
    if kernel == "dl_scatter":      # pre-word in, record out
        return 8 * S
    if kernel == "dl_first":        # records in, first position per code out, sorted first lists, bitmap
        return 4 * S + 4 * C + 8 * U + S // 8
    if kernel == "dl_fbscan":       # bitmap in, per-word prefix out
        return S // 8 + S // 16
    if kernel == "dl_ids":          # first positions in, two random rank reads per key, id per record out
        return 4 * C + 8 * S + 128 * U
    if kernel == "dl_words":        # record and id in (k_dl_ids' final word), the chunk's first-occurrence
        # bitmap in; word and the leaves out (no pre-word: rounds 2-5 charged 4 B per strand for one)
        return 12 * S + S // 8 + 8 * U
    if kernel == "flagscan_leaf":   # not-first marks; firsts: word, slot sector, leaf out, slot->id sector
        return S + U * (4 + 64 + 8 + 64 + 4)
    lv = list(zip(pk, layer_sizes))[:launches] if launches is not None else list(zip(pk, layer_sizes))
    if kernel == "flagscan_node":   # not-first marks, group records; firsts: pair re-read, node out, word
        return sum(p + 16 * ((p + 63) // 64) + u * (8 + 8 + 4 + 4) for p, u in lv)
    if kernel == "resolve_leaf":    # marks; non-first: word, slot->id sector, word
        return S + (S - U) * (4 + 64 + 4)
    if kernel == "resolve_node":    # marks; non-first: word in and out; the slot and group sectors
        # of the repeated keys (at most min(repeats, uniques) distinct keys, and no more lines
        # than the group array and the table hold: a hot key's repeats share its lines)
        return sum(p + (p - u) * (4 + 4) + min(128 * min(p - u, u), 16 * ((p + 63) // 64) + 8 * p) for p, u in lv)
    return 0


def dist_rank_bytes(kernel, L, Sr, r, R, c_r, u_r, n_leaves):
    """Algorithmic HBM bytes of one RANK's launches of `kernel` in a multi-rank build (the
    profiled rank r: Sr strands, pr = ceil(Sr / 2) layer-0 pairs, c_r leaves it holds first, u_r
    layer-0 uniques it emits; R ranks).  Streamed bytes + one 64-B sector per random access,
    like algorithmic_bytes, but over what this rank's launches touch: its own strands and pairs,
    the owner side's received records (~pr, owners balance by hash), the code-space passes over
    all 2^(2L-1) canonical codes and the R gathered presence bitmaps (gcz_dense.h, gcz_dist_fast.h).  Scopes
    without HBM work of their own (exchange, tail) count 0."""
    pr = (Sr + 1) // 2
    C = 2 ** (2 * L - 1)
    NB = dense_buckets(C)
    nch = (Sr + 32767) // 32768
    if kernel == "dl_pack":         # bases in, pre-word out, per-chunk bucket counts
        return Sr * L + 4 * Sr + 4 * NB * nch
    if kernel == "dl_scan":
        return 8 * NB * nch
    if kernel == "dl_scatter":      # pre-word in, record out
        return 8 * Sr
    if kernel == "dl_first":        # k_dl_first (records, first position per code, bitmap), the
        # r-first counts over the R gathered bitmaps, k_dl_rfirst (first positions, the lower
        # ranks' bitmaps, r-first lists), k_dl_fb (lists in, position bitmap out)
        return 4 * Sr + 8 * C + C // 8 + R * C // 8 + r * C // 8 + 12 * c_r + Sr // 8
    if kernel == "dl_fbscan":       # popcount scan; k_dl_gq: one rank lookup (a sector) per r-first code
        return Sr // 8 + Sr // 16 + 72 * c_r
    if kernel == "dl_ids":          # bitmaps of ranks <= r, relayed G reads per held code, record -> word
        return (r + 1) * C // 8 + 4 * min(n_leaves, Sr) + 8 * Sr + (Sr // 8 + 8 * c_r)
    if kernel == "dl_words":        # record, id in; word out
        return 12 * Sr + Sr // 8
    if kernel == "node_insert":     # k_node_keys: pre-word pairs in; canonical pair, word, marks out
        return 24 * pr
    if kernel == "dist_bucket":     # canonical pair, marks, word in; key and index out
        return 26 * pr
    if kernel == "dist_owner":      # ~pr received keys: partition, fine pass, LDS dedupe
        return 41 * pr
    if kernel == "dist_ids":        # reply flags -> global flags, look-ahead, the rank scan
        return 11 * pr
    if kernel == "dist_remap":
        return 8 * pr
    if kernel == "dist_l0":         # leaf word pairs, flags, ids in; words and unique nodes out
        return 17 * pr + 8 * u_r
    if kernel == "direct_levels":   # level-1 words in, the subtrees' nodes out (inner levels in LDS)
        return 12 * pr
    return 0


def build_bytes(L, S, n_leaves, layer_sizes):
    """Whole-build algorithmic bytes, SURVEY §8(d): B_stream + B_table."""
    pk = []
    n = S
    while True:
        p = (n + 1) // 2
        pk.append(p)
        if p == 1:
            break
        n = p
    b_stream = S * L + 4 * S + 8 * n_leaves + sum(4 * 2 * p + 4 * p + 8 * u for p, u in zip(pk, layer_sizes))
    b_table = 64 * (S + sum(pk))
    return b_stream, b_table


def traffic_file(config):
    """The newest round's PMC capture of a config: profiles/rNN/pmc_traffic_<config>.json with the
    highest NN (scripts/traffic_json.py writes it from the final evidence run of that round)."""
    import glob
    import re
    best = None
    for p in glob.glob(os.path.join(REPO, "profiles", "r*", f"pmc_traffic_{config}.json")):
        m = re.search(r"[/\\]r(\d+)[/\\]pmc_traffic_", p)
        if m and (best is None or int(m.group(1)) > best[0]):
            best = (int(m.group(1)), p)
    return best[1] if best else None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


class CpuBaseline:
    """Compiled reference (oracle/_ref/ref_harness, built from /root/reference sources)
    timed on this host: pack + shared_tree(std::vector<dna>&) build of the same synthetic
    genome, 1 thread (the reference builds single-threaded).  Started as a child process
    before the GPU work and joined at the end, so the full config fits the bench's wall
    time; it takes one host core of many."""

    def __init__(self, kind, nbases):
        self.kind, self.nbases, self.proc, self.t0 = kind, nbases, None, time.perf_counter()
        harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
        if os.path.exists(harness):
            self.proc = subprocess.Popen([harness, "time", str(kind), str(nbases), "12"], stdout=subprocess.PIPE,
                                         stderr=subprocess.PIPE, text=True)

    def result(self):
        host = f"{cpu_model()}, {os.cpu_count()} host CPUs visible, 1 used"
        sample = (f"synthetic {'uniform ACGT' if self.kind == 0 else 'tandem-repeat'} genome of the bench "
                  f"config (csrc/synth.h), all {self.nbases} bases, pack + build")
        if self.proc is not None:
            try:
                out, err = self.proc.communicate(timeout=900)
                if self.proc.returncode != 0:
                    raise RuntimeError(err.strip()[-300:])
                r = json.loads(out)
                return {"value": r["bases_per_s"], "unit": "bases/s", "cores": 1, "kind": "reference",
                        "sample": sample, "host": host, "build_ms": r["build_ms"], "pack_ms": r["pack_ms"],
                        "wall_s": round(time.perf_counter() - self.t0, 1)}
            except Exception as e:  # noqa: BLE001
                self.proc.kill()
                return {"value": None, "unit": "bases/s", "cores": 1, "kind": "reference", "error": str(e)}
        # port: the C restatement (test infrastructure) as the checker-side CPU timing, on a sample
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # noqa: E402
        gcz = sys.modules["gcz"]
        n = min(self.nbases, 120_000_000)
        data = gcz.synth(self.kind, n).tobytes()
        t0 = time.perf_counter()
        oracle.build_leaves(oracle.pack(data, 12), 12)
        dt = time.perf_counter() - t0
        return {"value": (len(data) // 12 * 12) / dt, "unit": "bases/s", "cores": 1, "kind": "port",
                "sample": f"first {n} bases of the bench genome, oracle/gcz_oracle.c", "host": host}


def stream_digest(group, dist, rank, world, info):
    """Bit identity of a distributed tree without assembling it: rank 0 hashes the
    ref_harness dump streams (leaves.bin; layers.bin = per layer a u64 node count and
    the raw words), taking the rank slices in rank order (rank r holds a contiguous id
    range of every layer) -- its own from HBM, the others' over gloo point-to-point."""
    layers = list(range(-1, info["n_layers"]))
    if world > 1:
        import torch   # already imported before libgcz when world > 1 (one HIP runtime)
    if rank != 0:
        for layer in layers:
            a = group.copy_slice(0, layer)
            dist.send(torch.tensor([a.size], dtype=torch.int64), 0)
            if a.size:
                dist.send(torch.from_numpy(a.view(np.int64) if layer < 0 else a.view(np.int32)), 0)
        return None
    h_leaves, h_layers = hashlib.sha256(), hashlib.sha256()
    for layer in layers:
        h = h_leaves if layer < 0 else h_layers
        if layer >= 0:
            h.update(np.uint64(info["layer_size"][layer]).astype("<u8").tobytes())
        for i in range(group.n_local):   # virtual ranks: every slice is local
            h.update(group.copy_slice(i, layer).tobytes())
        for src in range(1, world):
            n = torch.zeros(1, dtype=torch.int64)
            dist.recv(n, src)
            n = int(n.item())
            if n:
                t = torch.empty(n, dtype=torch.int64 if layer < 0 else torch.int32)
                dist.recv(t, src)
                h.update(t.numpy().tobytes())
    return {"sha_leaves_bin": h_leaves.hexdigest(), "sha_layers_bin": h_layers.hexdigest()}


LEAF_SCOPES = ("leaf_insert", "flagscan_leaf", "resolve_leaf", "dl_pack", "dl_probe", "dl_scan", "dl_scatter", "dl_first",
               "dl_fbscan", "dl_ids", "dl_words")


def rank_summary(rank, build_ms, trace, xlog=None):
    """One rank's profiled build: busy kernel time, exchange scopes (transfer + wait for the
    peers), host gaps, and when its leaf level ended (ms after the build's start event); with
    the group's exchange log (gcz_group_xlog), every collective's name and the bytes this rank
    sent to / received from the other ranks."""
    busy = sum(d for k, _, d in trace if k not in ("exchange", "mark"))
    xch = [(round(t, 3), round(d, 3)) for k, t, d in trace if k == "exchange"]
    leaf_end = max((t + d for k, t, d in trace if k in LEAF_SCOPES), default=None)
    x = sum(d for _, d in xch)
    out = {"rank": rank, "build_ms": round(build_ms, 3), "busy_ms": round(busy, 3), "exchange_ms": round(x, 3),
           "gap_ms": round(build_ms - busy - x, 3),
           "leaf_end_ms": round(leaf_end, 3) if leaf_end is not None else None, "exchanges": xch}
    if any(k == "mark" for k, _, _ in trace):
        # the fused schedule's compute segments (gcz_group::build_fast's fl_mark boundaries):
        # kernel time between consecutive marks, the last segment after the last mark
        segs, acc = [], 0.0
        for k, _, d in trace:
            if k == "mark":
                segs.append(round(acc, 4))
                acc = 0.0
            elif k != "exchange":
                acc += d
        out["segments_ms"] = segs + [round(acc, 4)]
    if xlog is not None:
        out["collectives"] = len(xlog)
        out["sent_bytes"] = sum(e["sent"] for e in xlog)
        out["recvd_bytes"] = sum(e["recvd"] for e in xlog)
        out["exchange_log"] = [[e["seq"], e["name"], e["sent"], e["recvd"]] for e in xlog]
    return out


def weak_run(gcz, ctx, group, dist, cfg, args, seed, L, world, rank, barrier):
    """Strong-scaled runs (the headline at N > 1) also time the weak-scaled case: one
    genome of N x the configured size, 1 config genome per GPU, on the same group."""
    import torch
    try:
        name = "uniform" if cfg["kind"] == 0 else "tandem"
        S1 = CONFIGS[args.config]["nbases"] * world // L
        golden = f"synth/{name}_{CONFIGS[args.config]['nbases'] * world}"
        a0, a1, _ = gcz.dist_plan(S1, world, rank)
        h1 = genome(gcz, cfg, seed, a0 * L, a1 * L)
        dev1 = ctx.upload(h1 if h1.size else np.zeros(1, np.uint8))
        del h1
        run1 = lambda: group.build_device_bases([dev1.ptr], S1, L)  # noqa: E731
        for _ in range(args.warmup):
            run1()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            i1 = run1()
        barrier()
        dt1 = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt1], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt1 = float(t.item())
        dev1.free()
        out = {"nbases": S1 * L, "per_gpu_nbases": S1 * L // world, "value": S1 * L * args.steps / dt1,
               "ms_per_step": dt1 / args.steps * 1e3, "device_ms": i1["build_ms"], "n_leaves": i1["n_leaves"],
               "scaling": "weak", "golden": golden}
        with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as f:
            exp = json.load(f).get(golden)
        if exp:
            out["layer_sizes_match"] = i1["layer_size"] == exp["expect"]["layer_sizes"]
            out["root_match"] = i1["root"] == exp["expect"]["root"]
        return out
    except Exception as e:  # noqa: BLE001 -- the weak line still prints
        return {"error": f"{type(e).__name__}: {e}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="uniform_1g", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--build-only", action="store_true",
                    help="skip the ratio path and decompression (PMC captures of the build alone)")
    ap.add_argument("--no-weak", action="store_true", help="strong runs at N > 1: skip the weak-scaled timing")
    ap.add_argument("--mode", choices=["weak", "strong", "dist", "replicas"], default="strong",
                    help="N > 1: the config genome itself over N GPUs (strong, the default; 'dist' is an alias), "
                         "one genome of N x the config size (weak), or N independent genomes (replicas)")
    ap.add_argument("--virtual", type=int, default=0, help="N = 1: distributed path with R virtual ranks")
    ap.add_argument("--rccl-world1", action="store_true", help="N = 1: the RCCL group path with one rank")
    ap.add_argument("--transport", choices=["rccl", "shm"], default="rccl",
                    help="N > 1 exchanges: RCCL over xGMI, or host-staged shared memory (several ranks on one GPU, "
                         "testing)")
    ap.add_argument("--shm-region-mb", type=int, default=1024)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        # A collective that never completes (a peer that died inside RCCL, a fabric
        # fault) would otherwise hold every rank until the launcher's own limit: after
        # GCZ_BENCH_WATCHDOG_S seconds each rank dumps all thread stacks to stderr and exits with status 1.
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ.get("GCZ_BENCH_WATCHDOG_S", "600")), exit=True)
        # CPU-side rendezvous only (barrier, max-over-ranks).  torch is imported
        # before libgcz so the process holds a single HIP runtime; no GPU tensor
        # or collective is on the build path.
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    gcz = load_gcz()
    cfg = CONFIGS[args.config]
    L = 12
    cpu_job = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cfg["kind"] != "file" and not args.virtual:
        cpu_job = CpuBaseline(cfg["kind"], cfg["nbases"])   # runs beside the GPU work
    if cfg["kind"] == "file":
        with open(os.path.join(REPO, cfg["path"]), "rb") as f:
            raw = f.read()
        cfg = dict(cfg, nbases=len(gcz.fasta_extract(raw)), file_size=len(raw))
    if args.mode == "dist":
        args.mode = "strong"
    weak = world > 1 and args.mode == "weak"
    if weak:   # one genome of world x the configured size, 1 config genome per GPU
        if cfg["kind"] == "file":
            sys.exit("--mode weak needs a synthetic config (the corpus files have a fixed size)")
        name = "uniform" if cfg["kind"] == 0 else "tandem"
        cfg = dict(cfg, nbases=cfg["nbases"] * world, golden=f"synth/{name}_{cfg['nbases'] * world}")
    nbases = cfg["nbases"]
    S = nbases // L
    mode = ("replicas" if args.mode == "replicas" else "dist") if world > 1 else ("virtual" if args.virtual else "single")
    if world == 1 and args.rccl_world1:
        mode = "dist"
    seed = gcz._lib.gcz_synth_default_seed()
    ctx = gcz.Context(local if args.transport == "rccl" else 0)   # shm: every rank on GPU 0
    group = None
    transport_used = "rccl" if args.transport == "rccl" else "shm"
    if mode == "dist":
        s0, s1, G = gcz.dist_plan(S, world, rank)
        host = genome(gcz, cfg, seed, s0 * L, s1 * L)
        dev = ctx.upload(host if host.size else np.zeros(1, np.uint8))
        if args.transport == "shm":   # testing: several ranks on one GPU, host-staged exchanges
            name = [f"/gcz_bench_{os.getpid()}_{time.time_ns()}" if rank == 0 else None]
            if dist is not None:
                dist.broadcast_object_list(name, src=0)
            group = gcz.Group.shm(ctx, rank, world, name[0], args.shm_region_mb << 20)
        else:
            uid = [gcz.dist_unique_id() if rank == 0 else None]
            if dist is not None:
                dist.broadcast_object_list(uid, src=0)
            err = None
            try:
                group = gcz.Group.rccl(ctx, rank, world, uid[0])
            except gcz.GczError as e:   # every rank learns of any rank's failure (gloo)
                err = str(e)
            failed = [err is not None]
            if dist is not None:
                flags = [None] * world
                dist.all_gather_object(flags, failed[0])
                failed = [any(flags)]
            if failed[0]:
                # RCCL could not form the communicator: the same build with host-staged
                # exchanges (correct, slower), labelled in the line ("transport") and the run
                # exits 4 -- it is not an RCCL number
                print(f"bench: RCCL group failed ({err}); falling back to the shm transport", file=sys.stderr)
                exit_code[0] = 4
                if group is not None:
                    group.close()
                name = [f"/gcz_bench_{os.getpid()}_{time.time_ns()}" if rank == 0 else None]
                if dist is not None:
                    dist.broadcast_object_list(name, src=0)
                group = gcz.Group.shm(ctx, rank, world, name[0], args.shm_region_mb << 20)
                transport_used = "shm (RCCL group creation failed)"
        prof_ctx = ctx
        run = lambda: group.build_device_bases([dev.ptr], S, L)  # noqa: E731
    elif mode == "virtual":
        group = gcz.Group.local(args.virtual, local)
        prof_ctx = group.ctx(0)
        host = genome(gcz, cfg, seed, 0, nbases)
        dev = prof_ctx.upload(host)
        ptrs = [dev.ptr + gcz.dist_plan(S, args.virtual, r)[0] * L for r in range(args.virtual)]
        run = lambda: group.build_device_bases(ptrs, S, L)  # noqa: E731
    else:
        if mode == "replicas":   # a different genome per rank, same size
            seed ^= 0 if rank == 0 else (0x5851F42D4C957F2D * rank) & ((1 << 64) - 1)
        host = genome(gcz, cfg, seed, 0, nbases)
        dev = ctx.upload(host)
        prof_ctx = ctx
        run = lambda: ctx.build_device_bases(dev.ptr, nbases, L)  # noqa: E731
    del host

    def barrier():
        prof_ctx.sync()
        if dist is not None:
            dist.barrier()
        prof_ctx.sync()

    for _ in range(args.warmup):
        run()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        info = run()
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    units = world * S * L if mode == "replicas" else S * L
    value = units * args.steps / dt

    # per-kernel device time (hipEvents on the library's launch stream), one extra build
    pctxs = [group.ctx(i) for i in range(group.n_local)] if mode == "virtual" else [prof_ctx]
    for c in pctxs:
        c.profile(True)
        c.profile_reset()
    barrier()   # ranks start the profiled build together: exchange waits are the peers' lag inside it
    info = run()
    tables = [c.profile_table() for c in pctxs]
    # N > 1: every rank's timeline of the profiled build (kernel busy time, exchanges incl. the
    # wait for peers, host gaps) -- where a rank waits is invisible in the max-over-ranks time
    rank_detail = None
    if mode == "dist":
        mine = rank_summary(rank, info["build_ms"], prof_ctx.profile_trace(), group.exchange_log(0))
        rank_detail = [mine]
        if dist is not None:
            rank_detail = [None] * world
            dist.all_gather_object(rank_detail, mine)
    elif mode == "virtual":
        rank_detail = [rank_summary(r, info["build_ms"], c.profile_trace(), group.exchange_log(r))
                       for r, c in enumerate(pctxs)]
    for c in pctxs:
        c.profile(False)
    prof = tables[0]
    rank_ms = [round(sum(v["total_ms"] for k, v in t.items() if k not in ("exchange", "mark")), 3) for t in tables]
    kernels = {}
    rank_model = None
    if mode in ("dist", "virtual"):   # the profiled rank's own launches (rank 0 of the virtual ranks)
        R = world if mode == "dist" else args.virtual
        me = rank if mode == "dist" else 0
        r0, r1, _ = gcz.dist_plan(S, R, me)
        rank_model = {"rank": me, "strands": r1 - r0, "pairs": (r1 - r0 + 1) // 2,
                      "first_leaves": group.slice(0, -1)[1], "layer0_uniques": group.slice(0, 0)[1]}
    for name, p in prof.items():
        if p["launches"] == 0 or name == "mark":
            continue
        if rank_model:
            b = dist_rank_bytes(name, L, rank_model["strands"], rank_model["rank"], R, rank_model["first_leaves"],
                                rank_model["layer0_uniques"], info["n_leaves"])
        else:
            b = algorithmic_bytes(name, L, S, info["n_leaves"], info["layer_size"], info["hashed_pairs"],
                                  info.get("bucketed_pairs", 0),
                                  two_pass=prof.get("bucket_fine", {}).get("launches", 0) > 0,
                                  launches=p["launches"], repetitive=bool(info.get("repetitive")))
        kernels[name] = {"launches": p["launches"], "total_ms": round(p["total_ms"], 4),
                         "avg_ms": p["total_ms"] / p["launches"], "alg_bytes": b,
                         "gbs": b / (p["total_ms"] * 1e-3) / 1e9 if p["total_ms"] > 0 else None}
    # the dominant kernel: the most device time among kernels that move algorithmic bytes
    dom = max((k for k in kernels if kernels[k]["alg_bytes"] > 0), key=lambda k: kernels[k]["total_ms"])
    dk = kernels[dom]
    # HBM bytes from the committed PMC capture of this config (scripts/traffic_json.py): per
    # build for each kernel name, and the whole build's
    traffic = None
    counter_build = None
    tpath = traffic_file(args.config)
    traffic_src = None
    if tpath and mode in ("single", "replicas"):
        with open(tpath) as f:
            tj = json.load(f)
        traffic_src = {"file": os.path.relpath(tpath, REPO), "code_head": tj.get("code_head")}
        per_build = tj.get("per_build", {})
        if dom in per_build:
            traffic = int(per_build[dom] / dk["launches"])
        counter_build = tj.get("build_total")
    roofline = {"bound": "hbm", "kernel": dom,
                "achieved": round(dk["alg_bytes"] / dk["launches"] / (dk["avg_ms"] * 1e-3) / 1e9, 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dk["alg_bytes"] / (dk["total_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                "traffic": traffic, "avg_launch_ms": round(dk["avg_ms"], 4),
                "alg_bytes_per_launch": dk["alg_bytes"] // dk["launches"]}
    b_stream, b_table = build_bytes(L, S, info["n_leaves"], info["layer_size"])
    build_frac = (b_stream + b_table) / (info["build_ms"] * 1e-3) / (HBM_PEAK_GBS * 1e9)
    counter_frac = (counter_build / (info["build_ms"] * 1e-3) / (HBM_PEAK_GBS * 1e9)) if counter_build else None

    parity = None
    tree = None
    golden = None
    with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as f:
        golden = json.load(f).get(cfg["golden"]) if cfg["golden"] else None
    exp = golden["expect"] if golden else None
    if not args.no_parity:
        if mode in ("dist", "virtual"):   # every rank streams its slices to rank 0
            t0 = time.perf_counter()
            d = stream_digest(group, dist, rank, world, info)
            if rank == 0:
                parity = {"golden": cfg["golden"] if exp else None, "digest_s": round(time.perf_counter() - t0, 2),
                          "layers_sha256": d["sha_layers_bin"], "leaves_sha256": d["sha_leaves_bin"]}
                if exp:
                    parity.update({"layers_sha256_match": d["sha_layers_bin"] == exp["sha_layers_bin"],
                                   "leaves_sha256_match": d["sha_leaves_bin"] == exp["sha_leaves_bin"],
                                   "root_match": info["root"] == exp["root"],
                                   "layer_sizes_match": info["layer_size"] == exp["layer_sizes"],
                                   "ratio_ref": exp["ratio"]})
                else:
                    parity["note"] = f"no reference golden for {cfg['golden']} (hashes reported)"
        elif rank == 0:                                            # replicas: rank 0 built the golden genome
            tree = ctx.tree()
    if tree is not None and (not exp or "sha_dag" not in exp):   # no golden: report the dump hashes
        parity = {"golden": None, "note": f"no reference golden for {cfg['golden']} (hashes reported)",
                  "leaves_sha256": hashlib.sha256(tree.leaves_bin()).hexdigest(),
                  "layers_sha256": hashlib.sha256(tree.layers_bin()).hexdigest()}
    elif tree is not None:
        d = gcz.digest(tree)
        ratio = f"{cfg.get('file_size', nbases) / d['bytes']:.6g}"   # compress reports file size / bytes()
        parity = {"golden": cfg["golden"],
                  "dag_sha256_match": d["sha_dag"] == exp["sha_dag"],
                  "unsorted_sha256_match": d["sha_unsorted_dag"] == exp["sha_unsorted_dag"],
                  "layers_sha256_match": d["sha_layers_bin"] == exp["sha_layers_bin"],
                  "ratio": ratio, "ratio_ref": exp["ratio"]}

    # ratio path on the device: frequency sort + bytes() + .dag writer
    ratio_path = None
    if mode in ("single", "replicas") and rank == 0 and not args.build_only:
        # a cold pass (first-call allocations), then the same pass timed on a fresh build
        n = gcz._U64()
        ctx.sync()
        t0 = time.perf_counter()
        ctx.sort_device()
        gcz._lib.gcz_device_dag(ctx._h, gcz.ctypes.byref(n))
        cold_ms = (time.perf_counter() - t0) * 1e3
        run()
        ctx.sync()
        t0 = time.perf_counter()
        ctx.sort_device()
        t1 = time.perf_counter()
        dptr = gcz._lib.gcz_device_dag(ctx._h, gcz.ctypes.byref(n))
        t2 = time.perf_counter()
        ratio_path = {"device_sort_ms": round((t1 - t0) * 1e3, 3), "device_dag_ms": round((t2 - t1) * 1e3, 3),
                      "cold_sort_dag_ms": round(cold_ms, 3),
                      "dag_bytes": int(n.value), "ratio": f"{cfg.get('file_size', nbases) / max(int(n.value), 1):.6g}"}
        if parity is not None:
            dag = ctx.serialize_device()
            parity["device_dag_sha256_match"] = exp is not None and hashlib.sha256(dag).hexdigest() == exp["sha_dag"]
        del dptr
        # decompression on the device (operator[] for every index) and the round trip
        text = ctx.upload(np.zeros(S * L, dtype=np.uint8))
        ctx.sync()
        t0 = time.perf_counter()
        rc = gcz._lib.gcz_decompress_device(ctx._h, gcz.ctypes.c_void_p(text.ptr), S * L)
        ratio_path["device_decompress_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        if rc == 0 and not args.no_parity:
            got = np.empty(S * L, dtype=np.uint8)
            gcz._lib.gcz_memcpy_d2h(ctx._h, gcz._ptr(got), gcz.ctypes.c_void_p(text.ptr), S * L)
            ref = genome(gcz, cfg, seed, 0, S * L)
            ratio_path["roundtrip_match"] = bool(np.array_equal(got, np.where(ref >= 97, ref - 32, ref)))
        text.free()

    # the distributed tree's ratio path on the device: every layer's rank slices
    # gathered device to device into one context on rank 0 (gcz_group_assemble), then its
    # frequency sort + bytes() + .dag writer -- no host gather, no host sort
    if mode in ("dist", "virtual") and not args.build_only:
        dst = gcz.Context(local if args.transport == "rccl" else 0) if rank == 0 else None
        try:
            if dist is not None:
                dist.barrier()
            prof_ctx.sync()
            t0 = time.perf_counter()
            group.assemble(dst)
            t1 = time.perf_counter()
            if rank == 0:
                n = gcz._U64()
                dst.sort_device()
                dst.sync()
                t2 = time.perf_counter()
                dptr = gcz._lib.gcz_device_dag(dst._h, gcz.ctypes.byref(n))
                dst.sync()
                t3 = time.perf_counter()
                del dptr
                ratio_path = {"assemble_ms": round((t1 - t0) * 1e3, 3), "device_sort_ms": round((t2 - t1) * 1e3, 3),
                              "device_dag_ms": round((t3 - t2) * 1e3, 3), "dag_bytes": int(n.value),
                              "ratio": f"{cfg.get('file_size', nbases) / max(int(n.value), 1):.6g}",
                              "note": "first call (cold): tree gathered to rank 0's device, sorted and written there"}
                if not args.no_parity and exp is not None and "sha_dag" in exp:
                    ratio_path["device_dag_sha256_match"] = hashlib.sha256(dst.serialize_device()).hexdigest() == exp["sha_dag"]
        except Exception as e:  # noqa: BLE001 -- reported in the line, the build numbers stand
            if rank == 0:
                ratio_path = {"error": f"{type(e).__name__}: {e}"}
        finally:
            if dst is not None:
                dst.close()

    weak_line = None
    if mode == "dist" and world > 1 and args.mode == "strong" and not args.no_weak and cfg["kind"] != "file":
        weak_line = weak_run(gcz, ctx, group, dist, cfg, args, seed, L, world, rank, barrier)

    cpu = cpu_job.result() if cpu_job is not None else None

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "bases/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak" if (args.mode in ("weak", "replicas") and mode != "virtual") else "strong",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "transport": transport_used if mode == "dist" else None,
            "config": {"workload": args.config, "nbases": nbases * (world if mode == "replicas" else 1),
                       "per_gpu_nbases": nbases // world if mode == "dist" else nbases, "L": L,
                       "strands": S * (world if mode == "replicas" else 1),
                       "parallelism": {"single": "1 GPU",
                                       "dist": f"dist{world}: one genome, strand ranges per GPU "
                                               f"({'1 config genome per GPU' if weak else 'config genome split'}), "
                                               f"owner-hashed all-to-all per level over {transport_used}",
                                       "replicas": f"{world} independent genomes, one per GPU",
                                       "virtual": f"{args.virtual} virtual ranks on 1 GPU (overhead probe)"}[mode]},
            "roofline": roofline,
            "build": {"device_ms": info["build_ms"], "hashed_pairs": info["hashed_pairs"],
                      "bucketed_pairs": info.get("bucketed_pairs", 0), "b_stream": b_stream, "b_table": b_table,
                      "hbm_frac_survey_formula": round(build_frac, 5),
                      # counter HBM bytes of a whole build (PMC capture) over this build's time
                      "counter_traffic_bytes": counter_build,
                      "counter_traffic_source": traffic_src,
                      "hbm_frac_counter": round(counter_frac, 5) if counter_frac else None,
                      "n_leaves": info["n_leaves"],
                      "n_layers": info["n_layers"],
                      # builds of the last step (> 1: a bucket / leaf-table overflow rebuilt it;
                      # device_ms is the last attempt, device_ms_all every attempt's)
                      "attempts": info.get("attempts", 1), "device_ms_all": info.get("build_ms_all")},
            "kernels": kernels,
            "rank_byte_model": rank_model,
            "rank_kernel_ms": rank_ms,
            "rank_timeline": rank_detail,
            "ratio_path": ratio_path,
            "cpu_baseline": cpu,
            "parity": parity,
            "weak_scaling": weak_line,
        }
        print(json.dumps(line), flush=True)
        bad = [k for src in (parity or {}, weak_line or {}) for k, v in src.items()
               if k.endswith("_match") and v is False]
        for k in ("roundtrip_match", "device_dag_sha256_match"):
            if ratio_path and ratio_path.get(k) is False:
                bad.append(k)
        if bad:
            print(f"bench: parity mismatch against the reference goldens: {bad}", file=sys.stderr, flush=True)
            exit_code[0] = 3
    dev.free()
    if group is not None:
        group.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


exit_code = [0]

if __name__ == "__main__":
    try:
        main()
        sys.exit(exit_code[0])
    except Exception as e:  # noqa: BLE001 -- report a failed run as a result line, not silence
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "bases/s",
                              "n_gpus": int(os.environ.get("WORLD_SIZE", "1")), "higher_is_better": True,
                              "error": f"{type(e).__name__}: {e}"}), flush=True)
        raise
