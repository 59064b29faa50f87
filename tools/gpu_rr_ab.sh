#!/bin/bash
# random_ray compaction (MCPT_RR_COMPACT) on the spill-free kernel at 7/6/5 waves vs main
export TMPDIR=/tmp; O=gpurun_out/${1:-rr_ab}; mkdir -p $O
MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_rr1w5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_rr1w5.log 2>&1; rc=$?
tail -1 $O/pytest_rr1w5.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libs_ab.sh ${1:-rr_ab} "6 8 3 1" 256 "2 4" main rr1w7 rr1w6 rr1w5
MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_stamps.so timeout -k 10 200 python tools/stamps.py > gpurun_out/${1:-rr_ab}/stamps.jsonl 2>&1
