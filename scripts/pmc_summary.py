#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs.

usage: pmc_summary.py <fetch_dir> <write_dir> [builds]
FETCH_SIZE / WRITE_SIZE are in KiB (x1024 -> bytes).  Calibration on this
machine (tools/microbench/atomics.hip, same rocprofv3): one random 8-B load
reads back ~64 B of FETCH_SIZE, one random CAS counts 64 B of WRITE_SIZE, so
for these random-access kernels the raw counters are used uncorrected.
Prints JSON: kernel -> {launches, fetch_bytes, write_bytes, traffic_per_launch}.
Round 2: the streaming kernels (dense leaf level, two-pass bucket partition) read
coalesced; on gfx950 FETCH_SIZE tallies a 128-B read request as 64 B
(MI355X_MICROARCH.md, HBM section), so `traffic_corrected_per_launch` doubles
FETCH_SIZE (2 x fetch + write) -- the figure bench.py reports for those kernels.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("gcz_dev::", "")
    m = re.match(r"(?:void )?([\w:]+)", name)
    return m.group(1) if m else name[:40]


NAMES = {"k_leaf_bases": "leaf_insert", "k_leaf_packed": "leaf_insert", "k_node_insert": "node_insert",
         "k_flagscan_leaf": "flagscan_leaf", "k_flagscan_node": "flagscan_node", "k_resolve_leaf": "resolve_leaf",
         "k_resolve_node": "resolve_node", "k_clear": "clear", "__amd_rocclr_fillBufferAligned": "clear",
         "k_tail": "tail", "k_direct_levels": "direct_levels", "k_dup_probe": "dl_probe",
         "k_dup_decide": "dl_probe", "k_bkt_count": "bucket_count", "k_bkt_scatter": "bucket_scatter",
         "k_bkt_dedupe": "bucket_dedupe", "k_bkt_part": "bucket_scatter", "k_bkt_fine": "bucket_fine",
         "k_bkt_dedupe2": "bucket_dedupe", "k_bkt_dedupe_bm": "bucket_dedupe", "k_bkt_dedupe2_redo": "bucket_dedupe",
         "k_build_init": "clear", "k_build_finish": "clear",
         "k_dl_pack": "dl_pack", "k_dl_scatter": "dl_scatter", "k_dl_first": "dl_first", "k_dl_fb": "dl_first",
         "k_dl_ids": "dl_ids", "k_dl_words": "dl_words"}


def load(d, counter):
    acc = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        k = NAMES.get(short(r["Kernel_Name"]), short(r["Kernel_Name"]))
        acc[k][0] += 1
        acc[k][1] += float(r["Counter_Value"]) * 1024
    return acc


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        n = max(f[k][0], w[k][0])
        out[k] = {"launches": n, "fetch_bytes": f[k][1], "write_bytes": w[k][1],
                  "traffic_per_launch": (f[k][1] + w[k][1]) / n if n else None,
                  "traffic_corrected_per_launch": (2 * f[k][1] + w[k][1]) / n if n else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
