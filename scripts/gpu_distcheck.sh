# Multi-rank path: virtual-rank tests, then weak-scaled virtual bench lines.
# usage: bash scripts/gpu_distcheck.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_dist_$tag.log 2>&1 &&
timeout -k 10 300 python bench.py --config uniform_2g --virtual 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/v2_$tag.log 2>&1 &&
timeout -k 10 400 python bench.py --config uniform_8g --virtual 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v8_$tag.log 2>&1
