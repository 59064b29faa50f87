#!/bin/bash
# Deep-BVH knobs on the current kernel: walk_exit x leaf_batch, 4 segments per item (AUTO's pick
# on scene 8), scenes 8 and 3.  tools/gpu_deep_sweep.sh OUTTAG
export TMPDIR=/tmp; O=gpurun_out/${1:-deep}; mkdir -p $O
for lb in 4 8 16; do
  MCPT_LEAF_BATCH=$lb MCPT_SEG_PER_ITEM=4 timeout -k 10 300 python tools/ab_time.py --scenes 8 3 --modes 1 --spp 256 \
    --walk-exit 8 16 24 32 --tag lb$lb >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
done
cat $O/sweep.jsonl
