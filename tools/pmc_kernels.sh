#!/bin/bash
# PMC passes over any command, one rocprofv3 run per counter group (never combined with the
# sys/runtime traces): tools/pmc_kernels.sh OUTDIR python3 tools/ab_time.py ...
# Summarise per kernel with tools/pmc_kernels.py OUTDIR.
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- "${CMD[@]}" > "$OUT/$name.log" 2>&1
}
CMD=("$@")
run sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
run sqb SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR
run sqc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_MISC
run tcc TCC_HIT_sum TCC_MISS_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
echo pmc done
