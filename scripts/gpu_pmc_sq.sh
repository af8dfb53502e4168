# One SQ-counter pass (8 counters) over bench.py --build-only of a config; per-kernel sums to
# gpurun_out/pmc_sq_<tag>.txt.   usage: bash scripts/gpu_pmc_sq.sh <tag> <config> "<C1 C2 ...>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; cfg=$2; ctrs=$3
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/pmc_$tag -o run -- python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only > gpurun_out/pmc_$tag.log 2>&1 || { tail -5 gpurun_out/pmc_$tag.log; exit 1; }
python3 - gpurun_out/pmc_$tag > gpurun_out/pmc_sq_$tag.txt <<'PY'
import csv, glob, sys, re
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(.*", "", r["Kernel_Name"])[:40]
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
names = sorted({c for v in agg.values() for c in v})
print("kernel".ljust(40), *[c[3:][:14].rjust(14) for c in names])
for n, v in sorted(agg.items(), key=lambda kv: -kv[1].get(names[0], 0)):
    print(n.ljust(40), *[f"{v.get(c, 0):14.4g}" for c in names])
PY
head -30 gpurun_out/pmc_sq_$tag.txt
