# Round-5 GPU batch: the fused multi-rank schedule's parity, then virtual-rank probes.
#   usage: bash scripts/gpu_r05.sh <tag> "<pytest args>" "<virtual probes: R:config ...>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; tests=$2; probes=$3
mkdir -p gpurun_out
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest $tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_${tag}_tests.txt 2>&1 || { tail -40 gpurun_out/r05_${tag}_tests.txt; exit 1; }
  tail -3 gpurun_out/r05_${tag}_tests.txt
fi
for pr in $probes; do
  R=${pr%%:*}; c=${pr#*:}
  o=gpurun_out/r05_${tag}_v${R}_${c}.json
  timeout -k 10 400 python bench.py --virtual $R --config $c --steps 3 --warmup 1 --no-cpu-baseline > $o 2>gpurun_out/r05_${tag}_v${R}_${c}.err || { tail -20 gpurun_out/r05_${tag}_v${R}_${c}.err; exit 1; }
  python - "$o" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k: round(v["total_ms"], 3) for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["total_ms"])[:10]}
print(sys.argv[1], round(d["ms_per_step"], 3), d["rank_kernel_ms"], ks, d.get("parity"))
print([e[1] for e in d["rank_timeline"][0]["exchange_log"]])
PY
done
