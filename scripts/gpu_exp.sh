# Kernel stats of one virtual-rank probe under several values of an environment knob (one
# rocprofv3 kernel-trace run each).  usage: bash scripts/gpu_exp.sh <VAR> "<v1 v2 ...>" [R] [config] [kernel regex]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
var=$1; vals=$2; R=${3:-8}; cfg=${4:-uniform_8g}; pat=${5:-k_fl_|k_dl_|k_bkt_|k_ob_}
mkdir -p gpurun_out/exp
for v in $vals; do
  export "$var=$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp/d$v -o d$v -- python3 bench.py --virtual $R --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only > gpurun_out/exp/d$v.json 2> gpurun_out/exp/d$v.err || { tail -20 gpurun_out/exp/d$v.err; exit 1; }
  db=$(find gpurun_out/exp/d$v -name '*.db' | head -1)
  echo "$var=$v"; python3 scripts/rocpd_kernels.py "$db" --stats | grep -E "$pat" | head -20
  rm -rf gpurun_out/exp/d$v
done
