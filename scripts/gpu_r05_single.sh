# Round-5 single-GPU probe: the default config's bench line and rocprof kernel stats, the
# tandem config's bench line.  usage: bash scripts/gpu_r05_single.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-s}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_${tag}_bench.json 2> gpurun_out/r05_${tag}_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_${tag}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/r05_${tag}_prof.log 2>&1 &&
timeout -k 10 300 python bench.py --config tandem_3g2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05_${tag}_tandem.json 2> gpurun_out/r05_${tag}_tandem.err
