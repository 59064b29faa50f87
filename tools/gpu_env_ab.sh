#!/bin/bash
# A/B of one environment knob of the default library: parity suites at the first value, then
# per-lane timings and launch-shape costs at every value.
#   tools/gpu_env_ab.sh TAG VAR "scenes" v1 v2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; VAR=$2; SCENES=$3; shift 3
mkdir -p $O
export $VAR=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py \
  tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$1.log 2>&1 ||
  { echo "parity FAILED at $VAR=$1"; tail -30 $O/pytest_$1.log; exit 1; }
tail -1 $O/pytest_$1.log
for v in "$@"; do
  export $VAR=$v
  timeout -k 10 300 python tools/ab_time.py --scenes $SCENES --modes 1 --tag $VAR=$v \
    >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  timeout -k 10 300 python tools/launch_shape_cost.py > $O/shape_$v.jsonl 2>&1 || exit $?
done
cat $O/ab.jsonl
for v in "$@"; do echo "== $VAR=$v"; grep '^{' $O/shape_$v.jsonl; done
