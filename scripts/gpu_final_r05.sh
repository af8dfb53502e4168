# Round-5 evidence at HEAD: full GPU suite + smoke, the default bench (CPU baseline
# included), the rocprof / PMC passes of uniform_1g and tandem (part 1); the tandem and
# corpus bench lines, strong virtual-rank probes (uniform 8/4/2, tandem 8), the weak-scaled
# probe (8 Gbase over 8 virtual ranks = 1 Gbase per rank), the drop-in latency probe (part 2).
# usage: bash scripts/gpu_final_r05.sh <tag> [1|2|all]   (one gpurun call per part fits its limit)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r05f}; part=${2:-all}
mkdir -p gpurun_out
if [ "$part" = 1 ] || [ "$part" = all ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$tag.txt 2>&1 &&
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/pytest_gpu_$tag.txt 2>&1 &&
  timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err &&
  bash scripts/gpu_evidence.sh uniform_1g $tag &&
  bash scripts/gpu_evidence.sh tandem_3g2 $tag || exit $?
fi
if [ "$part" = 2 ] || [ "$part" = all ]; then
  timeout -k 10 300 python bench.py --config tandem_3g2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_tandem_$tag.json 2> gpurun_out/bench_tandem_$tag.err &&
  timeout -k 10 120 python bench.py --config merged --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_merged_$tag.json 2> gpurun_out/bench_merged_$tag.err &&
  timeout -k 10 120 python bench.py --config hehcmv --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_hehcmv_$tag.json 2> gpurun_out/bench_hehcmv_$tag.err || exit $?
  for R in 8 4 2; do
    timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v$R.json 2> gpurun_out/strong_${tag}_v$R.err || exit $?
  done
  timeout -k 10 300 python bench.py --virtual 8 --mode strong --config tandem_3g2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v8_tandem.json 2> gpurun_out/strong_${tag}_v8_tandem.err &&
  timeout -k 10 600 python bench.py --virtual 8 --mode strong --config uniform_8g --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/weak_${tag}_v8.json 2> gpurun_out/weak_${tag}_v8.err &&
  bash scripts/gpu_dropin_latency.sh $tag || exit $?
fi
