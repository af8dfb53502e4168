# Multi-rank node levels without the local dedupe: parity (virtual ranks, incl. the
# large goldens) and per-rank kernel time against the local-dedupe schedule.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/nolocal
mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_dist.py -m gpu -x -v -p no:cacheprovider > $O/pytest_dist.log 2>&1 || exit 1
for mode in 0 1; do
  for v in 2 8; do
    GCZ_DIST_LOCAL=$mode timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --virtual $v > $O/bench_v${v}_m${mode}.log 2>&1 || exit 1
  done
  GCZ_DIST_LOCAL=$mode timeout -k 10 300 python bench.py --config tandem_3g2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --virtual 8 > $O/bench_t_v8_m${mode}.log 2>&1 || exit 1
done
