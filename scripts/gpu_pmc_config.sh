# PMC traffic + kernel stats of one bench config (BASELINE config 3: data/merged).
# usage: bash scripts/gpu_pmc_config.sh <config> <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
cfg=${1:-merged}; tag=${2:-r01}
mkdir -p gpurun_out
B="python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-parity"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_${cfg}_$tag -o run -- $B > gpurun_out/pmc_fetch_${cfg}_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_${cfg}_$tag -o run -- $B > gpurun_out/pmc_write_${cfg}_$tag.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${cfg}_$tag -o run -- $B > gpurun_out/prof_${cfg}_$tag.log 2>&1 &&
timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${cfg}_$tag.log 2>&1
