#!/usr/bin/env python3
"""Per-kernel achieved HBM GB/s: PMC traffic (FETCH_SIZE + WRITE_SIZE runs) over the
kernel time of a separate --kernel-trace run of the same command.

usage: pmc_gbs.py <fetch_dir> <write_dir> <trace_dir>
"""
import csv
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import NAMES, load, short  # noqa: E402


def main(fetch, write, trace):
    f, w = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    dur = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f"{trace}/run_kernel_trace.csv")):
        k = NAMES.get(short(r["Kernel_Name"]), short(r["Kernel_Name"]))
        dur[k][0] += 1
        dur[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k in sorted(set(f) | set(w)):
        launches = f.get(k, [0, 0])[0] or w.get(k, [0, 0])[0]
        traffic = f.get(k, [0, 0.0])[1] + w.get(k, [0, 0.0])[1]
        n, t = dur.get(k, [0, 0.0])
        per_launch = traffic / launches if launches else 0.0
        out[k] = {"launches": launches, "traffic_per_launch": per_launch,
                  "avg_launch_s": t / n if n else None,
                  "achieved_gbs": per_launch / (t / n) / 1e9 if n and t else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
