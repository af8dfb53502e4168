# Single-GPU bench under table-size knobs: usage bash scripts/gpu_knobs.sh <tag> "ENV=.. ENV=.." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  env $kv timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/knob_${tag}_$i.log 2>&1 || exit 1
  echo "$kv" >> gpurun_out/knob_${tag}_$i.log
  i=$((i+1))
done
