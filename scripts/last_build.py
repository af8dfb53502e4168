#!/usr/bin/env python3
"""Per-kernel totals of the last build in a rocprofv3 kernel trace (from the last k_dup_probe
pair of a 2-virtual-rank run, or the last k_dup_probe of a single-rank run)."""
import csv
import re
import sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nrank = int(sys.argv[2]) if len(sys.argv) > 2 else 2


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    m = re.match(r"(?:void )?([\w:<>, ]+?)\(", n)
    return (m.group(1) if m else n[:50]).replace("gcz_dev::", "")


idx = [i for i, r in enumerate(rows) if "k_dup_probe" in r["Kernel_Name"]]
start = idx[-nrank]
agg = OrderedDict()
for r in rows[start:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg.setdefault(short(r["Kernel_Name"]), [0, 0.0])
    a[0] += 1
    a[1] += d
tot = sum(v[1] for v in agg.values())
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:50s} {n:5d} {t / nrank:9.1f} us/rank")
print(f"{'total':50s} {'':5s} {tot / nrank:9.1f} us/rank")
