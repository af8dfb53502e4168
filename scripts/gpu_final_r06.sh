# Round-6 evidence at one code HEAD.  Part 1: the FETCH/WRITE split captures of uniform_1g and
# tandem_3g2 (copied into profiles/r06 on the box first, so the bench lines below carry this
# code's counter bytes), the full GPU suite + smoke, the default bench (CPU baseline included)
# and its rocprofv3 kernel stats, the tandem bench and its kernel stats.  Part 2: the corpus bench
# lines, the virtual-rank probes (strong 8/4/2, tandem 8, weak 8 x 1 Gbase) with kernel stats of
# the strong R = 8 and weak probes, the drop-in latency probe.
# usage: bash scripts/gpu_final_r06.sh <tag> <code_head> [1|2|all]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r06f}; head=${2:-unknown}; part=${3:-all}
mkdir -p gpurun_out profiles/r06
if [ "$part" = 1 ] || [ "$part" = all ]; then
  bash scripts/gpu_pmc_split.sh ${tag}_u uniform_1g $head &&
  bash scripts/gpu_pmc_split.sh ${tag}_t tandem_3g2 $head &&
  cp gpurun_out/pmc_split_${tag}_u.json profiles/r06/pmc_traffic_uniform_1g.json &&
  cp gpurun_out/pmc_split_${tag}_t.json profiles/r06/pmc_traffic_tandem_3g2.json &&
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$tag.txt 2>&1 &&
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/pytest_gpu_$tag.txt 2>&1 &&
  timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_u_$tag -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_u_$tag.log 2>&1 &&
  timeout -k 10 300 python bench.py --config tandem_3g2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_tandem_$tag.json 2> gpurun_out/bench_tandem_$tag.err &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_t_$tag -o run -- python bench.py --config tandem_3g2 --steps 3 --warmup 1 --no-cpu-baseline --build-only > gpurun_out/prof_t_$tag.log 2>&1 || exit $?
fi
if [ "$part" = 2 ] || [ "$part" = all ]; then
  timeout -k 10 120 python bench.py --config merged --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_merged_$tag.json 2> gpurun_out/bench_merged_$tag.err &&
  timeout -k 10 120 python bench.py --config hehcmv --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_hehcmv_$tag.json 2> gpurun_out/bench_hehcmv_$tag.err || exit $?
  for R in 8 4 2; do
    timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v$R.json 2> gpurun_out/strong_${tag}_v$R.err || exit $?
  done
  timeout -k 10 300 python bench.py --virtual 8 --mode strong --config tandem_3g2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v8_tandem.json 2> gpurun_out/strong_${tag}_v8_tandem.err &&
  timeout -k 10 600 python bench.py --virtual 8 --mode strong --config uniform_8g --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/weak_${tag}_v8.json 2> gpurun_out/weak_${tag}_v8.err &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v8_$tag -o run -- python3 bench.py --virtual 8 --config uniform_1g --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only > gpurun_out/prof_v8_$tag.log 2>&1 &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w8_$tag -o run -- python3 bench.py --virtual 8 --config uniform_8g --steps 2 --warmup 1 --no-cpu-baseline --no-parity --build-only > gpurun_out/prof_w8_$tag.log 2>&1 &&
  bash scripts/gpu_dropin_latency.sh $tag || exit $?
  find gpurun_out/prof_*_$tag -name '*kernel_trace.csv' -o -name '*kernel_stats.csv' | head -20
fi
