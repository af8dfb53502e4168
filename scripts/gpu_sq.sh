# SQ counters of the bench's kernels (SQ_ARGS: extra bench arguments, e.g. --config merged) (two passes of <= 8 SQ counters, --kernel-trace beside)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-sq}
mkdir -p gpurun_out
B="python bench.py ${SQ_ARGS:---steps 1 --warmup 1} --no-cpu-baseline --no-parity"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/sq1_$tag -o run -- $B > gpurun_out/sq1_$tag.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/sq2_$tag -o run -- $B > gpurun_out/sq2_$tag.log 2>&1
