set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cal
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/cal/p -o run --output-format csv -- ./tools/microbench/lane_util > gpurun_out/cal/log 2>&1
