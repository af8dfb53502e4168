# Full GPU test suite + default bench + tandem 3.2G bench, each step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -x -v -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_uv.log 2>&1 &&
GCZ_PROFILE_VERBOSE=1 timeout -k 10 300 python bench.py --config tandem_3g2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_t32.log 2> gpurun_out/bench_t32.err
