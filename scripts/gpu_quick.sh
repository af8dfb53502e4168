# quick sanity: smoke + short bench; usage: bash scripts/gpu_quick.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-quick}; shift || true
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bench_$tag.log 2>&1
