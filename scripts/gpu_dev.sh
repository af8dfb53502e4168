# dev loop: a pytest subset then a short bench; usage: bash scripts/gpu_dev.sh <tag> "<pytest -k expr>" [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-dev}; k=${2:-dense}; shift 2 || true
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "$k" > gpurun_out/pytest_$tag.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bench_$tag.log 2>&1
