# Rank 0's share of the strands (GCZ_DIST_RANK0_PERMILLE) on R virtual ranks: per-rank kernel
# time for each setting.  usage: bash scripts/gpu_share.sh <tag> "<R:permille ...>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
for rp in $2; do
  R=${rp%%:*}; pm=${rp##*:}
  o=gpurun_out/share_${tag}_${R}_$pm.json
  GCZ_DIST_RANK0_PERMILLE=$pm timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline --no-parity --build-only > $o 2>&1 || { tail -5 $o; exit 1; }
  python -c "import json,sys; d=json.loads(open('$o').read().strip().splitlines()[-1]); print('R=$R pm=$pm', d['rank_kernel_ms'], max(d['rank_kernel_ms']))"
done
