# Round evidence at HEAD: GPU tests, smoke, default bench, then the rocprof/PMC passes.
# usage: bash scripts/gpu_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$tag.txt 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/pytest_gpu_$tag.txt 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err &&
bash scripts/gpu_evidence.sh uniform_1g $tag
