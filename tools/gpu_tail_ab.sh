#!/bin/bash
# Segment groups x grid-tail fill: parity at (3, 2), then per-lane timings at 256 spp for each
# "K:TAIL" pair (MCPT_SEG_PER_ITEM, MCPT_TAIL_ROUNDS).  tools/gpu_tail_ab.sh TAG "scenes" K:T ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; SCENES=$2; shift 2
mkdir -p $O
export MCPT_SEG_PER_ITEM=3 MCPT_TAIL_ROUNDS=2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_full_size.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 ||
  { echo "parity FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for kt in "$@"; do
  export MCPT_SEG_PER_ITEM=${kt%%:*} MCPT_TAIL_ROUNDS=${kt##*:}
  timeout -k 10 300 python tools/ab_time.py --scenes $SCENES --modes 1 --spp 256 --reps 2 --tag $kt \
    >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
cat $O/ab.jsonl
