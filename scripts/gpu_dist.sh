# Multi-rank path on one GPU: virtual-rank parity (incl. 100 Mbase), RCCL world-1,
# full GPU suite, and bench lines for single / virtual ranks / RCCL world 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_dist.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider --deselect tests/test_dist.py > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_single.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --rccl-world1 > gpurun_out/bench_rccl1.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --virtual 2 > gpurun_out/bench_v2.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --virtual 8 > gpurun_out/bench_v8.log 2>&1
