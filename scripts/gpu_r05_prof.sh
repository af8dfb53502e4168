# rocprofv3 kernel trace of one virtual-rank probe: bash scripts/gpu_r05_prof.sh <tag> <R> <config>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; R=$2; c=$3
mkdir -p gpurun_out/r05p
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05p/$tag -o $tag -- python3 bench.py --virtual $R --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only > gpurun_out/r05p/$tag.json 2> gpurun_out/r05p/$tag.err || { tail -20 gpurun_out/r05p/$tag.err; exit 1; }
db=$(find gpurun_out/r05p/$tag -name '*.db' | head -1)
python3 scripts/rocpd_kernels.py "$db" --stats > gpurun_out/r05p/${tag}_stats.txt
python3 scripts/rocpd_kernels.py "$db" --build 700 > gpurun_out/r05p/${tag}_seq.txt
rm -f "$db"
head -25 gpurun_out/r05p/${tag}_stats.txt
