# Virtual-rank probes (strong 1 Gbase at R = 8 / 4 / 2, weak 8 Gbase over 8) into gpurun_out/probe_<tag>_*.json
# usage: bash scripts/gpu_probe_r06.sh <tag> [R list] [weak 0|1]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; Rs=${2:-"8 4 2"}; weak=${3:-1}
mkdir -p gpurun_out
for R in $Rs; do
  timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/probe_${tag}_v$R.json 2> gpurun_out/probe_${tag}_v$R.err || { tail -5 gpurun_out/probe_${tag}_v$R.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/probe_${tag}_v$R.json').read().strip().splitlines()[-1])
print('R=$R', 'rank kernels', d['rank_kernel_ms'], 'parity', {k:v for k,v in (d.get('parity') or {}).items() if k.endswith('match')})"
done
if [ "$weak" = 1 ]; then
  timeout -k 10 600 python bench.py --virtual 8 --mode strong --config uniform_8g --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/probe_${tag}_w8.json 2> gpurun_out/probe_${tag}_w8.err || { tail -5 gpurun_out/probe_${tag}_w8.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/probe_${tag}_w8.json').read().strip().splitlines()[-1])
print('weak R=8', 'rank kernels', d['rank_kernel_ms'], 'parity', {k:v for k,v in (d.get('parity') or {}).items() if k.endswith('match')})"
fi
