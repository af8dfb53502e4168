# Round-end evidence: smoke, full GPU suite, default bench (CPU baseline included),
# rocprofv3 kernel stats of the same command, PMC traffic passes, tandem config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-final}
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$tag.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/prof_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- $B > gpurun_out/pmc_fetch_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$tag -o run -- $B > gpurun_out/pmc_write_$tag.log 2>&1 &&
GCZ_PROFILE_VERBOSE=1 timeout -k 10 300 python bench.py --config tandem_3g2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_t32_$tag.log 2> gpurun_out/bench_t32_$tag.err
