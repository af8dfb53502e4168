# Weak-scaled distributed path, virtual ranks: 8 x 1 Gbase bench line (hashes) and a
# rocprofv3 kernel trace of 2 x 1 Gbase.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config uniform_8g --virtual 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/weak_virtual_8g.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v2 -o run -- python bench.py --config uniform_2g --virtual 2 --steps 1 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/prof_v2.log 2>&1
