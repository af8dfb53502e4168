#!/usr/bin/env python3
"""Print the headline and per-kernel-group times of bench.py result lines."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    if d.get("error"):
        print(f, "ERROR", d["error"])
        continue
    p = d.get("parity") or {}
    ok = {k: v for k, v in p.items() if k.endswith("match")}
    print(f"{f}: {d['value'] / 1e9:.1f} Gbase/s  {d['ms_per_step']:.3f} ms/step  rank_ms={d.get('rank_kernel_ms')}  {ok}")
    print("   " + "  ".join(f"{k}={v['total_ms']:.3f}" for k, v in d["kernels"].items()))
