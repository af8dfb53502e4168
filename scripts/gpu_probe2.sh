set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/probe_teardown.py > gpurun_out/probe_td1.log 2>&1; echo "td1=$?" >> gpurun_out/probe_td1.log
timeout -k 10 120 python scripts/probe_teardown.py --profile > gpurun_out/probe_td2.log 2>&1; echo "td2=$?" >> gpurun_out/probe_td2.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --virtual 2 > gpurun_out/bench_v2.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --virtual 8 > gpurun_out/bench_v8.log 2>&1
