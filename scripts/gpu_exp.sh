# Experiment batch on one MI355X: parity subset, A/B of env knobs on bench configs, a virtual-rank
# profile.  usage: bash scripts/gpu_exp.sh <tag> "<pytest files>" "<knob sets>" "<configs>"
#   knob sets: space-separated, each comma-joined VAR=VAL list ("-" = defaults)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; tests=$2; knobs=${3:--}; cfgs=${4:-uniform_1g}
mkdir -p gpurun_out
if [ -n "$tests" ]; then
  timeout -k 10 600 python -u -m pytest $tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/exp_${tag}_tests.txt 2>&1 || { tail -30 gpurun_out/exp_${tag}_tests.txt; exit 1; }
  tail -1 gpurun_out/exp_${tag}_tests.txt
fi
for c in $cfgs; do
  for kv in $knobs; do
    env_args=$( [ "$kv" = "-" ] && echo "" || echo "$kv" | tr ',' ' ')
    o=gpurun_out/exp_${tag}_${c}_$(echo "$kv" | tr ',=' '_-').json
    env $env_args timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --build-only --no-parity > $o 2>&1 || { tail -5 $o; exit 1; }
    python - "$o" "$kv" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k: round(v["total_ms"], 3) for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["total_ms"])[:8]}
print(sys.argv[3], sys.argv[2], round(d["ms_per_step"], 3), d["rank_kernel_ms"], ks)
PY
  done
done
