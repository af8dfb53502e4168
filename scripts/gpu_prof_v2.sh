# rocprofv3 kernel trace of the distributed path with 2 virtual ranks on 2 x 1 Gbase.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v2_$tag -o run -- python bench.py --config uniform_2g --virtual 2 --steps 1 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/prof_v2_$tag.log 2>&1
