# Drop-in first-tree latency on the box: the reference CLI (oracle/_ref/ref_compress, CPU) and
# ours on data/merged, the init probe's phase split, and `compress` on 1 Gbase with phase lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
G=genome-compression_amd
o=gpurun_out/dropin_${1:-r03}.txt
test -x tools/probe/init_probe || /opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude tools/probe/init_probe.cpp -L$G -lgcz \
  -Wl,-rpath,'$ORIGIN/../../genome-compression_amd' -o tools/probe/init_probe || exit $?
test -x oracle/_ref/ref_compress || { echo "oracle/_ref/ref_compress missing (make -C oracle ref)"; exit 2; }
: > $o
for i in 1 2 3; do
  echo "## ref_compress merged $i" >> $o
  timeout -k 10 120 oracle/_ref/ref_compress --statistics --output=/tmp/merged_ref.dag tests/golden/data/merged >> $o 2>&1 || exit $?
  echo "## compress merged $i" >> $o
  GCZ_TIMING=1 timeout -k 10 120 $G/compress --statistics --output=/tmp/merged.dag tests/golden/data/merged >> $o 2>&1 || exit $?
done
sha256sum /tmp/merged_ref.dag /tmp/merged.dag >> $o &&
echo "## init_probe merged" >> $o &&
timeout -k 10 120 tools/probe/init_probe tests/golden/data/merged >> $o 2>&1 &&
timeout -k 10 120 $G/gen_synth 0 1000000000 /tmp/u1g.txt &&
for i in 1 2; do
  echo "## compress u1g $i" >> $o
  GCZ_TIMING=1 timeout -k 10 300 $G/compress --statistics --output=/tmp/u1g.dag /tmp/u1g.txt >> $o 2>&1 || exit $?
done
sha256sum /tmp/u1g.dag >> $o
