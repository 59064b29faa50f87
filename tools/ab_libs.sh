#!/bin/bash
# Kernel A/B timing over library variants: tools/ab_libs.sh OUTTAG "scenes" lib1 lib2 ...
# (libmcpt_<name>.so under montecarlo-pathtracing_amd/mcpt/variants; per-lane walk)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; SCENES=$2; shift 2
mkdir -p $O
for w in "$@"; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$w.so timeout -k 10 300 \
    python tools/ab_time.py --scenes $SCENES --modes 1 --tag $w >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
