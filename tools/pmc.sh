#!/bin/bash
# PMC passes on the bench workload (one rocprofv3 run per counter group; --pmc never
# combined with sys/runtime traces).  Usage: tools/pmc.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
# warm-up steps; the summary reads the timed step's launch (bench.py runs AUTO's timing trials first)
# (PMC_STEPS timed steps: pmc_summary.py --calls=PMC_STEPS averages their launches)
ARGS="--steps ${PMC_STEPS:-1} --warmup 2 --no-cpu-baseline --no-count --no-check $*"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
run sqb SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR
run sqc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU
if [ -n "$PMC_MEM" ]; then   # memory hierarchy of the gathers (mesh workload): L1 -> L2 requests and
  # their latency, L2 hits / misses, fabric requests by size and the DRAM share of them
  run tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
  run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
  run tcc2 TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_REQ_sum
  run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
fi
echo pmc done
