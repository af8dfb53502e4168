# A/B of two builds of libgcz on the default bench (per-kernel times from the line's hipEvent
# profile): ab/libgcz_base.so (a saved earlier build) against the tree's libgcz.so, two runs each.
# usage: bash scripts/gpu_lib_ab.sh <tag> [bench args]; AB_EXTRA="x y" also runs ab/libgcz_x.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
lib=genome-compression_amd/libgcz.so
cp $lib /tmp/libgcz_new.so
for v in base new $AB_EXTRA; do
  if [ $v = new ]; then cp /tmp/libgcz_new.so $lib; else cp ab/libgcz_$v.so $lib; fi
  for rep in 1 2; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --build-only "$@" > gpurun_out/lab_${tag}_${v}_$rep.json 2> gpurun_out/lab_${tag}_${v}_$rep.err || { tail -5 gpurun_out/lab_${tag}_${v}_$rep.err; cp /tmp/libgcz_new.so $lib; exit 1; }
    python3 - "$v" gpurun_out/lab_${tag}_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = sorted(d["kernels"].items(), key=lambda kv: -kv[1]["total_ms"])
par = d.get("parity") or {}
print(f"[{sys.argv[1]}] ms/step {d['ms_per_step']:.4f} device {d['build']['device_ms']:.4f} parity {all(v for k, v in par.items() if k.endswith('_match'))} | " +
      " ".join(f"{k}={v['total_ms']:.4f}" for k, v in ks[:12]))
PY
  done
done
cp /tmp/libgcz_new.so $lib
