# Distributed-level depth sweep (GCZ_DIST_TAIL_LOG2) on virtual ranks: tandem 3.2G over 8, uniform 8 x 1G
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 9 14 17 20; do
  GCZ_DIST_TAIL_LOG2=$t timeout -k 10 300 python bench.py --config tandem_3g2 --virtual 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tail_t32_$t.log 2>&1 || exit 1
done
for t in 9 17; do
  GCZ_DIST_TAIL_LOG2=$t timeout -k 10 300 python bench.py --config uniform_8g --virtual 8 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/tail_u8_$t.log 2>&1 || exit 1
done
