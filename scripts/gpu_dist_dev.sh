# multi-rank dev loop: dist tests then the virtual strong probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-dd}; shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_dist.py "$@" > gpurun_out/pytest_dist_$tag.log 2>&1 &&
for R in 8 2; do
  timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v$R.log 2> gpurun_out/strong_${tag}_v$R.err || exit $?
done
