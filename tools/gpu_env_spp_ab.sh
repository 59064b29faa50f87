#!/bin/bash
# Per-lane timings of the default library at several values of one environment knob, at a given
# pass count per launch:  tools/gpu_env_spp_ab.sh TAG VAR SPP "scenes" v1 v2 ...
# (value "auto" leaves VAR unset)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; VAR=$2; SPP=$3; SCENES=$4; shift 4
mkdir -p $O
for v in "$@"; do
  if [ "$v" = auto ]; then unset $VAR; else export $VAR=$v; fi
  timeout -k 10 300 python tools/ab_time.py --scenes $SCENES --modes 1 --spp $SPP --reps 2 --tag $VAR=$v \
    >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
