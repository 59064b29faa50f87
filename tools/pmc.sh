#!/bin/bash
# PMC passes on the bench workload (one rocprofv3 run per counter group; --pmc never
# combined with sys/runtime traces).  Usage: tools/pmc.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
# warm-up steps; the summary reads the timed step's launch (bench.py runs AUTO's timing trials first)
ARGS="--steps 1 --warmup 2 --no-cpu-baseline --no-count --no-check $*"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
run sqb SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR
run sqc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU
echo pmc done
