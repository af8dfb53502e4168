# Round evidence for one bench config from one HEAD: rocprofv3 kernel trace + stats of the
# default bench command, and FETCH_SIZE / WRITE_SIZE passes (separate runs, no trace
# domains) of the build alone.  usage: bash scripts/gpu_evidence.sh <config> <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
cfg=${1:-uniform_1g}; tag=${2:-r03}
mkdir -p gpurun_out
B="python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity --build-only"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev_prof_${cfg}_$tag -o run -- python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ev_prof_${cfg}_$tag.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/ev_fetch_${cfg}_$tag -o run -- $B > gpurun_out/ev_fetch_${cfg}_$tag.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/ev_write_${cfg}_$tag -o run -- $B > gpurun_out/ev_write_${cfg}_$tag.log 2>&1
