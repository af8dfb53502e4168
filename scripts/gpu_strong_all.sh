# strong-scaling probes on one GPU at HEAD: the 1 Gbase genome over 2 / 4 / 8 virtual ranks,
# the 3.2 Gbase tandem genome over 8, and the multi-process (shm) tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-sa}
mkdir -p gpurun_out
for R in 8 4 2; do
  timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/strong_${tag}_v$R.log 2> gpurun_out/strong_${tag}_v$R.err || exit $?
done
timeout -k 10 300 python bench.py --config tandem_3g2 --virtual 8 --mode strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_t8.log 2> gpurun_out/strong_${tag}_t8.err &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_multiproc.py > gpurun_out/pytest_mp_$tag.log 2>&1
