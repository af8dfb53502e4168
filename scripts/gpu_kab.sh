# Kernel-level A/B: rocprofv3 kernel traces of a short bench with the default library and
# with each variant exp/<name>/libgcz.so; usage: bash scripts/gpu_kab.sh "<name> ..." [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
v=$1; shift
mkdir -p gpurun_out
L=genome-compression_amd/libgcz.so
cp $L /tmp/libgcz_base.so || exit 1
rc=0
for n in base $v; do
  if [ $n != base ]; then cp exp/$n/libgcz.so $L || { rc=1; break; }; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kab_$n -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity "$@" > gpurun_out/kab_$n.log 2>&1 || { rc=$?; break; }
done
cp /tmp/libgcz_base.so $L; exit $rc
