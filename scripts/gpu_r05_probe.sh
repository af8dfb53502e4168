set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c/v8 -o v8 -- python3 bench.py --virtual 8 --config uniform_1g --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only > gpurun_out/r05c/v8.json 2> gpurun_out/r05c/v8.err || { tail -20 gpurun_out/r05c/v8.err; exit 1; }
timeout -k 10 600 python3 bench.py --virtual 8 --config uniform_8g --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05c/w8.json 2> gpurun_out/r05c/w8.err || { tail -20 gpurun_out/r05c/w8.err; exit 1; }
ls -R gpurun_out/r05c | head -30
