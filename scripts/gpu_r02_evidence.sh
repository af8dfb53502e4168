# Round-2 evidence of the default bench: rocprofv3 kernel stats, and FETCH_SIZE /
# WRITE_SIZE passes (one counter per run, --kernel-trace only beside it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r02}
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/prof_$tag.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- $B > gpurun_out/pmc_fetch_$tag.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$tag -o run -- $B > gpurun_out/pmc_write_$tag.log 2>&1
