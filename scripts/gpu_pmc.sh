# PMC passes (one counter group per run, --kernel-trace only alongside, per MI355X guide)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r01}
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- $B > gpurun_out/pmc_fetch_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$tag -o run -- $B > gpurun_out/pmc_write_$tag.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_fetch_$tag -o run -- ./tools/microbench/atomics > gpurun_out/pmc_cal_fetch_$tag.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_cal_write_$tag -o run -- ./tools/microbench/atomics > gpurun_out/pmc_cal_write_$tag.log 2>&1 &&
timeout -k 10 900 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_full_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full_$tag -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/prof_full_$tag.log 2>&1
