# Weak-scaled distributed path, 8 virtual ranks (8 x 1 Gbase on one MI355X): rocprofv3
# kernel trace of one build (per-rank kernel costs at R = 8) and the plain bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config uniform_8g --virtual 8 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/weak_v8.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v8 -o run -- python bench.py --config uniform_8g --virtual 8 --steps 1 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/prof_v8.log 2>&1
