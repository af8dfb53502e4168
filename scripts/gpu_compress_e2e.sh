# End-to-end `compress --statistics` (file read + build + sort + .dag write) on the box,
# next to the compiled reference's compress timing from BASELINE.md.  GCZ_TIMING=1 phase
# lines on stderr; the second 1 Gbase run uses the runtime's pageable copy for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
G=genome-compression_amd
timeout -k 10 120 $G/gen_synth 0 1000000000 /tmp/u1g.txt &&
GCZ_TIMING=1 timeout -k 10 300 $G/compress --statistics --output=/tmp/u1g.dag /tmp/u1g.txt > gpurun_out/compress_u1g.csv 2>&1 &&
sha256sum /tmp/u1g.dag >> gpurun_out/compress_u1g.csv &&
GCZ_TIMING=1 GCZ_UPLOAD=pageable timeout -k 10 300 $G/compress --statistics --output=/tmp/u1g.dag /tmp/u1g.txt > gpurun_out/compress_u1g_pageable.csv 2>&1 &&
GCZ_TIMING=1 timeout -k 10 300 $G/compress --statistics --output=/tmp/u1g.dag /tmp/u1g.txt > gpurun_out/compress_u1g_2.csv 2>&1 &&
timeout -k 10 300 $G/compress --statistics --output=/tmp/merged.dag tests/golden/data/merged > gpurun_out/compress_merged.csv 2>&1 &&
sha256sum /tmp/merged.dag >> gpurun_out/compress_merged.csv
