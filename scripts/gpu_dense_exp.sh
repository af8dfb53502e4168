# dense leaf level experiments (timing only); usage: bash scripts/gpu_dense_exp.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-dx}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k dense > gpurun_out/pytest_$tag.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_${tag}_a.log 2>&1 &&
GCZ_DENSE_NB=1024 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_${tag}_b.log 2>&1 &&
GCZ_DENSE_EXP=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_${tag}_c.log 2>&1
