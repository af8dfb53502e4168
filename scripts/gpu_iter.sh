# Iteration check: dist + parity GPU tests, the 8-virtual-rank weak line (with rank
# timelines), and single-device bench lines for a knob sweep given as "VAR=v1,v2".
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-it}
timeout -k 10 600 python -u -m pytest tests/test_dist.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1 &&
timeout -k 10 300 python bench.py --config uniform_8g --virtual 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/v8_$tag.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/b1_$tag.log 2>&1 || exit 1
if [ -n "$2" ]; then
  var=${2%%=*}; vals=${2#*=}
  for v in ${vals//,/ }; do
    env $var=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/b1_${tag}_${var}_$v.log 2>&1 || exit 1
  done
fi
