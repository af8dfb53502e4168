# FETCH_SIZE and WRITE_SIZE passes (separate runs) of bench.py --build-only on a config, then the
# per-kernel read (2 x FETCH) / write split per build (scripts/traffic_json.py) into
# gpurun_out/pmc_split_<tag>.json.   usage: bash scripts/gpu_pmc_split.sh <tag> <config> [code_head]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; cfg=$2; head=${3:-}
mkdir -p gpurun_out
B="python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pf_$tag -o run -- $B > gpurun_out/pf_$tag.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pw_$tag -o run -- $B > gpurun_out/pw_$tag.log 2>&1 || { tail -5 gpurun_out/pf_$tag.log gpurun_out/pw_$tag.log; exit 1; }
fd=$(dirname $(find gpurun_out/pf_$tag -name '*counter_collection.csv' | head -1))
wd=$(dirname $(find gpurun_out/pw_$tag -name '*counter_collection.csv' | head -1))
cd scripts && python3 traffic_json.py ../$fd ../$wd $cfg ../gpurun_out/pmc_split_$tag.json $head && cd .. &&
rm -rf gpurun_out/pf_$tag gpurun_out/pw_$tag
