#!/usr/bin/env python3
"""profiles/traffic_<config>.json from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE captures of
`bench.py --config <config> --build-only` (scripts/gpu_evidence.sh): HBM bytes per build
for each of bench.py's kernel names and for the whole build.

usage: traffic_json.py <fetch_dir> <write_dir> <config> <out.json> [code_head]
(out.json: profiles/rNN/pmc_traffic_<config>.json -- bench.py reads the newest round's)
Every launch in the capture belongs to a build (--build-only); builds are counted by
k_build_init (one per build attempt).  gfx950 correction (MI355X_MICROARCH.md, HBM /
rocprofv3 section): FETCH_SIZE tallies a 128-B read request as 64 B, so a kernel's bytes
are 2 x FETCH_SIZE + WRITE_SIZE (both in KiB).
"""
import csv
import json
import sys
from collections import defaultdict

from pmc_summary import NAMES, short

EXTRA = {"k_scan_excl": "scan", "k_seg_expand": "node_insert", "k_tail": "tail",
         "__amd_rocclr_copyBuffer": "copy"}


def load(d, counter):
    """Bytes per kernel name over the dispatches from the first build on (k_build_init): the
    bench's setup before it -- the upload of the bases and its first-touch fill of 1 GB -- is not
    a build's traffic (rounds 3-5 spread it over the builds as 200-250 MB of "clear")."""
    acc = defaultdict(float)
    inits = 0
    rows = [r for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")) if r["Counter_Name"] == counter]
    key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else None
    if key:
        rows.sort(key=lambda r: int(r[key]))
    started = key is None
    for r in rows:
        s = short(r["Kernel_Name"])
        if s == "k_build_init":
            inits += 1
            started = True
        if not started:
            continue
        k = NAMES.get(s, EXTRA.get(s.split("<")[0], s))
        acc[k] += float(r["Counter_Value"]) * 1024
    return acc, inits


def main():
    f, nf = load(sys.argv[1], "FETCH_SIZE")
    w, nw = load(sys.argv[2], "WRITE_SIZE")
    builds = max(1, min(nf, nw))
    keys = sorted(set(f) | set(w))
    per = {k: round((2 * f[k] + w[k]) / builds) for k in keys}
    out = {"config": sys.argv[3], "code_head": sys.argv[5] if len(sys.argv) > 5 else None,
           "builds": builds, "per_build": per, "build_total": sum(per.values()),
           # the two sides apart: read bytes (2 x FETCH_SIZE) and written bytes (WRITE_SIZE)
           "per_build_read": {k: round(2 * f[k] / builds) for k in keys},
           "per_build_write": {k: round(w[k] / builds) for k in keys},
           "_note": "HBM bytes per build from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of "
                    "bench.py --build-only (scripts/gpu_evidence.sh), 2 x FETCH_SIZE + WRITE_SIZE "
                    "(gfx950: FETCH_SIZE tallies a 128-B read as 64 B)"}
    with open(sys.argv[4], "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps({"builds": builds, "build_total": out["build_total"]}))


if __name__ == "__main__":
    main()
