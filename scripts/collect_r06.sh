# Copy one round-6 evidence capture from gpurun_out/ into profiles/r06/ (runs here, no GPU).
# usage: bash scripts/collect_r06.sh <part-1 tag> <part-2 tag>
set -eo pipefail
cd "$(dirname "$0")/.."
a=$1; b=$2; o=gpurun_out; d=profiles/r06
mkdir -p $d
last() { grep '^{' "$1" | tail -1 > "$2"; }
cp $o/pmc_split_${a}_u.json $d/pmc_traffic_uniform_1g.json
cp $o/pmc_split_${a}_t.json $d/pmc_traffic_tandem_3g2.json
cp $o/pytest_gpu_$a.txt $d/pytest_gpu.txt
last $o/bench_$a.json $d/bench.json
last $o/bench_tandem_$a.json $d/bench_tandem_3g2.json
python3 scripts/prof_summary.py $o/prof_u_$a/run_kernel_trace.csv > $d/rocprof_summary.txt
cp $o/prof_u_$a/run_kernel_stats.csv $d/rocprof_kernel_stats.csv
python3 scripts/prof_summary.py $o/prof_t_$a/run_kernel_trace.csv > $d/rocprof_summary_tandem_3g2.txt
cp $o/prof_t_$a/run_kernel_stats.csv $d/rocprof_kernel_stats_tandem_3g2.csv
last $o/bench_merged_$b.json $d/bench_merged.json
last $o/bench_hehcmv_$b.json $d/bench_hehcmv.json
for R in 2 4 8; do last $o/strong_${b}_v$R.json $d/strong_virtual$R.json; done
last $o/strong_${b}_v8_tandem.json $d/strong_virtual8_tandem_3g2.json
last $o/weak_${b}_v8.json $d/weak_virtual8_uniform_8g.json
python3 scripts/prof_summary.py $o/prof_v8_$b/run_kernel_trace.csv > $d/rocprof_strong_virtual8_stats.txt
python3 scripts/prof_summary.py $o/prof_w8_$b/run_kernel_trace.csv > $d/rocprof_weak_virtual8_uniform_8g_stats.txt
cp $o/dropin_$b.txt $d/compress_e2e.txt
ms=$(python3 -c "import json;print(round(json.load(open('$d/bench.json'))['ms_per_step'],4))")
mt=$(python3 -c "import json;print(round(json.load(open('$d/bench_tandem_3g2.json'))['ms_per_step'],4))")
{
  echo "# scripts/budget.py on the round-6 virtual-rank probes (profiles/r06, capture $b)."
  echo "# single-GPU ms per Gbase = bench.json ms_per_step ($ms ms, capture $a); tandem: bench_tandem_3g2.json ($mt ms)."
  echo "# latency 25 us per collective and t_sync 15 us per host round trip are ASSUMED (RCCL at world > 1 has not run here)."
  for R in 8 4 2; do echo; echo "## strong, 1 Gbase, R = $R"; python3 scripts/budget.py $d/strong_virtual$R.json $ms; done
  echo; echo "## weak, 8 Gbase over 8 ranks"; python3 scripts/budget.py $d/weak_virtual8_uniform_8g.json $ms --weak
  echo; echo "## strong, 3.2 Gbase tandem, R = 8"; python3 scripts/budget.py $d/strong_virtual8_tandem_3g2.json $mt
} > $d/exchange_budget.txt
ls $d
