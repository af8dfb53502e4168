# bench + per-kernel rocprofv3 trace (csv) ; usage: bash scripts/gpu_bench.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-run}; shift || true
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_$tag.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bench_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity "$@" > gpurun_out/prof_$tag.log 2>&1
