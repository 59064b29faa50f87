#!/bin/bash
# A/B of the per-wave unit pool: K segments per work item (MCPT_SEG_PER_ITEM), new library
# against a baseline variant.  tools/gpu_pool_ab.sh OUTTAG BASELINE_VARIANT "scenes" SPP
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; BASE=$2; SCENES=$3; SPP=${4:-256}
mkdir -p $O
for k in 1 2 4 8; do
  MCPT_SEG_PER_ITEM=$k timeout -k 10 300 python tools/ab_time.py --scenes $SCENES --modes 1 --spp $SPP \
    --tag new_K$k >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
for k in 1 2 4; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$BASE.so MCPT_SEG_PER_ITEM=$k timeout -k 10 300 \
    python tools/ab_time.py --scenes $SCENES --modes 1 --spp $SPP --tag ${BASE}_K$k >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
