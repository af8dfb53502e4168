# rocprofv3 kernel stats of a short bench; usage: bash scripts/gpu_prof.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-prof}; shift || true
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity "$@" > gpurun_out/prof_$tag.log 2>&1
