# strong-scaling probe on one GPU: the 1 Gbase genome over R virtual ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-sp}; shift || true
mkdir -p gpurun_out
for R in 8 2; do
  timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/strong_${tag}_v$R.log 2> gpurun_out/strong_${tag}_v$R.err || exit $?
done
