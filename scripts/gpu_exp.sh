set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for v in 16 17 18 24 50 59; do
  export GCZ_FL_DBG=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp/d$v -o d$v -- python3 bench.py --virtual 8 --config uniform_8g --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only > gpurun_out/exp/d$v.json 2> gpurun_out/exp/d$v.err || { tail -20 gpurun_out/exp/d$v.err; exit 1; }
  db=$(find gpurun_out/exp/d$v -name '*.db' | head -1)
  echo "dbg=$v"; python3 scripts/rocpd_kernels.py "$db" --stats | grep -E "k_fl_scatter"
  rm -rf gpurun_out/exp/d$v
done
