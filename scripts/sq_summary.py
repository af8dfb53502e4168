#!/usr/bin/env python3
"""Per-kernel SQ counter totals from scripts/gpu_sq.sh runs (summed over the build's
dispatches of each kernel): usage sq_summary.py <dir> [<dir> ...]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("gcz_dev::", "")
    m = re.match(r"(?:void )?([\w:]+)", name)
    return m.group(1) if m else name[:40]


acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k:22s} n={len(disp[k]):3d} wait={c.get('SQ_WAIT_ANY',0)/wc:5.2f} stall={c.get('SQ_WAIT_INST_ANY',0)/wc:5.2f} "
          f"active={c.get('SQ_ACTIVE_INST_ANY',0)/wc:5.2f} valu={c.get('SQ_ACTIVE_INST_VALU',0)/wc:5.2f} "
          f"lds={c.get('SQ_ACTIVE_INST_LDS',0)/wc:5.2f} vmem={c.get('SQ_ACTIVE_INST_VMEM',0)/wc:5.2f} "
          f"insts_valu={c.get('SQ_INSTS_VALU',0):.3g} lds={c.get('SQ_INSTS_LDS',0):.3g} rd={c.get('SQ_INSTS_VMEM_RD',0):.3g} "
          f"wr={c.get('SQ_INSTS_VMEM_WR',0):.3g} bankc={c.get('SQ_LDS_BANK_CONFLICT',0):.3g} waves={c.get('SQ_WAVES',0):.3g}")
