#!/bin/bash
# GPU session: variant libraries (montecarlo-pathtracing_amd/mcpt/variants/libmcpt_<v>.so) —
# the parity suite on each, then per-lane-walk timing.  tools/gpu_variant_ab.sh TAG "scenes" v1 v2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; SCENES=$2; shift 2
mkdir -p $O
for v in "$@"; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$v.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q -k "not sharded" --timeout 300 --timeout-method thread \
    > $O/pytest_$v.log 2>&1 || { echo "variant $v parity FAILED"; tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for v in "$@"; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$v.so timeout -k 10 300 \
    python tools/ab_time.py --scenes $SCENES --modes 1 --tag $v >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
