# Multi-rank check on one MI355X: the distributed-path tests, then the per-rank cost on R
# virtual ranks (bench.py --virtual R) for R = 8 4 2 and the tandem config at R = 8.
# usage: bash scripts/gpu_dist_check.sh <tag> [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-dev}; k=${2:-}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist.py tests/test_multiproc.py tests/test_bench_digest.py -m gpu -x -q \
  --timeout 200 --timeout-method thread ${k:+-k "$k"} > gpurun_out/dist_$tag.txt 2>&1 || { tail -30 gpurun_out/dist_$tag.txt; exit 1; }
tail -2 gpurun_out/dist_$tag.txt
for R in 8 4 2; do
  timeout -k 10 300 python bench.py --virtual $R --mode strong --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v$R.json 2> gpurun_out/strong_${tag}_v$R.err || exit $?
done
timeout -k 10 300 python bench.py --virtual 8 --mode strong --config tandem_3g2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/strong_${tag}_v8_tandem.json 2> gpurun_out/strong_${tag}_v8_tandem.err || exit $?
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"strong_{t}_v8", f"strong_{t}_v4", f"strong_{t}_v2", f"strong_{t}_v8_tandem"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    par = d.get("parity") or {}
    print(f, d.get("rank_kernel_ms"), {k: v for k, v in par.items() if k.endswith("match")})
PY
