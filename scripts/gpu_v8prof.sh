# virtual-rank strong-scaling probe: per-scope verbose timing + rocprof kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-v8}; R=${2:-8}; shift 2 || true
mkdir -p gpurun_out
GCZ_PROFILE_VERBOSE=1 timeout -k 10 300 python bench.py --virtual $R --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${tag}.log 2> gpurun_out/${tag}.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --virtual $R --steps 2 --warmup 1 --no-cpu-baseline --no-parity "$@" > gpurun_out/prof_$tag.log 2>&1
