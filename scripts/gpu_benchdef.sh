# the driver's default bench line + the multi-process (shm) strong/weak test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-bd}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_multiproc.py > gpurun_out/pytest_mp_$tag.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench_def_$tag.log 2> gpurun_out/bench_def_$tag.err
