#!/bin/bash
# Launch-shape cost (tools/launch_shape_cost.py) for each variant library:
#   tools/gpu_shape_ab.sh TAG v1 v2 ...   (montecarlo-pathtracing_amd/mcpt/variants/libmcpt_<v>.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for v in "$@"; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$v.so timeout -k 10 300 \
    python tools/launch_shape_cost.py > $O/shape_$v.jsonl 2>&1 || exit $?
  echo "== $v"; grep '^{' $O/shape_$v.jsonl
done
