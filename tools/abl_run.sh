#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/abl1; mkdir -p $O
for w in base abl_fastmath abl_fasttrans abl_cheaphash abl_norr2 abl_allabl abl_allablw; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$w.so timeout -k 10 300 \
    python tools/ab_time.py --scenes 6 8 --modes 1 --tag $w >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
