#!/bin/bash
# Kernel A/B over libraries x segment groups (per-lane walk, AUTO's LANE candidates):
#   tools/gpu_libs_ab.sh OUTTAG "scenes" SPP "K list" lib1 lib2 ...
# lib "main" = the in-tree libmcpt.so, others = variants/libmcpt_<name>.so.  Interleaved by K
# so that the libraries see the same box state.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; SCENES=$2; SPP=$3; KS=$4; shift 4
mkdir -p $O
for k in $KS; do
  for w in "$@"; do
    if [ "$w" = main ]; then L=montecarlo-pathtracing_amd/mcpt/libmcpt.so; else L=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$w.so; fi
    MCPT_LIB=$L MCPT_SEG_PER_ITEM=$k timeout -k 10 300 python tools/ab_time.py --scenes $SCENES --modes 1 \
      --spp $SPP --tag ${w}_K$k >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  done
done
cat $O/ab.jsonl
