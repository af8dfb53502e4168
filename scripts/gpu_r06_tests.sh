# usage: bash scripts/gpu_r06_tests.sh <tag> "<pytest args>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/tests_$tag.txt 2>&1
rc=$?
tail -5 gpurun_out/tests_$tag.txt
exit $rc
