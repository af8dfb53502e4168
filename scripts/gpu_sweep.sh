# env-knob sweep of bench.py (no tests); usage: bash scripts/gpu_sweep.sh tag "ENV=.. ENV=.." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/sweep_${tag}_$i.log 2>&1 || exit 1
  echo "$cfg" > gpurun_out/sweep_${tag}_$i.cfg
  i=$((i+1))
done
