# Sliced leaf translation A/B (virtual ranks, 2 x 1 Gbase)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 0 -1 4 16; do
  GCZ_XLATE_PASSES=$p timeout -k 10 300 python bench.py --config uniform_2g --virtual 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xlate_$p.log 2>&1 || exit 1
done
