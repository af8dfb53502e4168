# Weak-scaled genomes (N x 1 Gbase) on one GPU: the single-device build (hashes /
# golden parity) and the distributed path with N virtual ranks (per-rank kernel time).
# usage: bash scripts/gpu_weak.sh "2 4 8"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${1:-2 4 8}; do
  timeout -k 10 400 python bench.py --config uniform_${n}g --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/weak_single_${n}g.log 2>&1 &&
  timeout -k 10 400 python bench.py --config uniform_${n}g --virtual $n --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/weak_virtual_${n}g.log 2>&1 || exit 1
done
