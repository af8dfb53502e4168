#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace csv: per kernel calls / total / avg (us),
and the per-dispatch durations of the last build (in launch order)."""
import csv
import re
import sys
from collections import OrderedDict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void )?([\w:<>, ]+?)\(", name)
    return m.group(1) if m else name[:60]


def main(path, per_build=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    agg = OrderedDict()
    for r in rows:
        k = short(r["Kernel_Name"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':40s} {'calls':>6s} {'total_us':>11s} {'avg_us':>9s} {'share':>6s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:40s} {n:6d} {t:11.1f} {t / n:9.2f} {100 * t / tot:5.1f}%")
    if per_build:
        last = rows[-per_build:]
        print("\nlast build, dispatch order:")
        for r in last:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"  {short(r['Kernel_Name']):40s} grid={r['Grid_Size_X']:>10s} {d:9.1f} us  vgpr={r['VGPR_Count']}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
