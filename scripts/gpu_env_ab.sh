# A/B of environment settings on the default bench (per-kernel times from the line's hipEvent
# profile).  usage: bash scripts/gpu_env_ab.sh <tag> "<ENV=v ENV2=v>" "<ENV=v>" ... [-- bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
i=0
for s in "${sets[@]}"; do
  for rep in 1 2; do
    env $s timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --build-only "$@" > gpurun_out/ab_${tag}_${i}_$rep.json 2> gpurun_out/ab_${tag}_${i}_$rep.err || { tail -5 gpurun_out/ab_${tag}_${i}_$rep.err; exit 1; }
    python3 - "$s" gpurun_out/ab_${tag}_${i}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = sorted(d["kernels"].items(), key=lambda kv: -kv[1]["total_ms"])
par = d.get("parity") or {}
print(f"[{sys.argv[1]}] ms/step {d['ms_per_step']:.4f} device {d['build']['device_ms']:.4f} parity {all(v for k, v in par.items() if k.endswith('_match'))} | " +
      " ".join(f"{k}={v['total_ms']:.4f}" for k, v in ks[:14]))
PY
  done
  i=$((i+1))
done
