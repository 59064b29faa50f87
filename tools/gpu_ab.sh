#!/bin/bash
# GPU session: parity tests, then kernel A/B over occupancy variants × traversal modes.
#   tools/gpu_ab.sh OUTTAG "scenes" "variants"
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
SCENES=${2:-"6 8 1 3"}
VARS=${3:-"w4 w5 w6"}
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for w in $VARS; do
  # parity of the variant itself (bit-exact vs the oracle) before timing it
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$w.so timeout -k 10 600 \
    python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "scene_parity or event_counters or full_hd" \
    > $O/pytest_$w.log 2>&1 || { echo "variant $w parity FAILED"; tail -20 $O/pytest_$w.log; exit 1; }
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$w.so timeout -k 10 300 \
    python tools/ab_time.py --scenes $SCENES --modes 1 2 --tag $w >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
