# Multi-process (shm transport) bench test on one GPU, then the full GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -x -v -p no:cacheprovider --timeout 300 > gpurun_out/pytest_mp_$tag.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --deselect tests/test_multiproc.py > gpurun_out/pytest_gpu_$tag.log 2>&1
