#!/bin/bash
# Per-lane timings of variant libraries under one environment setting, at a given pass count:
#   tools/gpu_lib_env_ab.sh TAG "VAR=VALUE" SPP "scenes" lib1 lib2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; ENVSET=$2; SPP=$3; SCENES=$4; shift 4
mkdir -p $O
export "$ENVSET"
for w in "$@"; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$w.so timeout -k 10 300 \
    python tools/ab_time.py --scenes $SCENES --modes 1 --spp $SPP --reps 2 --tag "$w $ENVSET" >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
