# dense + dist tests, single bench, virtual strong probes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-ad}; shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_dist.py -k "dense or dist" > gpurun_out/pytest_$tag.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 &&
for R in 8 2; do
  timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v$R.log 2> gpurun_out/strong_${tag}_v$R.err || exit $?
done
