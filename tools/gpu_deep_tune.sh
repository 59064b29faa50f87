#!/bin/bash
# Deep-BVH kernel knobs re-check: walk_exit sweep at several leaf_batch values (MCPT_LEAF_BATCH)
# on the deep scenes, per-lane walk, 256 spp launches.  tools/gpu_deep_tune.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for lb in 4 8 16; do
  export MCPT_LEAF_BATCH=$lb
  timeout -k 10 400 python tools/ab_time.py --scenes 8 3 7 --modes 1 --spp 256 --reps 1 \
    --walk-exit 8 16 24 32 --tag leaf_batch=$lb >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
