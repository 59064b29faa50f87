#!/bin/bash
# GPU tests, then three default bench runs (AUTO's pick and run-to-run spread): tools/gpu_bench3.sh TAG
export TMPDIR=/tmp; O=gpurun_out/${1:-bench3}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-count >> $O/bench3.jsonl 2>> $O/bench3.err || exit 1
done
python - "$O/bench3.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["value"], d["kernel_ms"]["trace_avg"], d["self_check"]["bit_equal"])
PY
