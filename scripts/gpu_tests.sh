# run a subset of the GPU tests: usage: bash scripts/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-t}; shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu "$@" > gpurun_out/pytest_$tag.log 2>&1
