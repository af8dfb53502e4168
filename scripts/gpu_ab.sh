# A/B of the default library against a variant built under exp/<name>/libgcz.so (bench only)
# usage: bash scripts/gpu_ab.sh "<name> <name> ..." [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
v=$1; shift
mkdir -p gpurun_out
L=genome-compression_amd/libgcz.so
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/ab_base.log 2>&1 &&
cp $L /tmp/libgcz_base.so || exit 1
rc=0
for n in $v; do
  cp exp/$n/libgcz.so $L &&
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/ab_$n.log 2>&1 || { rc=$?; break; }
done
cp /tmp/libgcz_base.so $L; exit $rc
