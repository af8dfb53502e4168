# Alternating A/B of two environment settings on the default bench's timed steps (no profile):
# A B A B A B, 30 steps each.  usage: bash scripts/gpu_ab_alt.sh <tag> "<ENV=a>" "<ENV=b>" [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; a=$2; b=$3; shift 3
mkdir -p gpurun_out
for i in 1 2 3; do
  for s in "$a" "$b"; do
    env $s timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --build-only "$@" > gpurun_out/alt_${tag}.json 2> gpurun_out/alt_${tag}.err || { tail -5 gpurun_out/alt_${tag}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/alt_${tag}.json').read().strip().splitlines()[-1])
print('[$s] ms/step %.4f' % d['ms_per_step'])"
  done
done
