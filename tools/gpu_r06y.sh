#!/bin/bash
# round 6 session y: pass stealing inside a wave (MCPT_STEAL=1, variant build `steal`): the mesh
# full-size parity tests under it, then interleaved timing against main with stealing on and off
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06y2}; mkdir -p $O
MCPT_STEAL=1 MCPT_LIB=$PWD/montecarlo-pathtracing_amd/mcpt/variants/libmcpt_steal.so timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py -k "mesh" -x -q --timeout 300 --timeout-method thread > $O/pytest_steal.log 2>&1; rc=$?; echo "pytest steal rc=$rc"; tail -3 $O/pytest_steal.log; [ $rc -eq 0 ] || exit $rc
MCPT_STEAL=1 timeout -k 10 400 python tools/ab_interleave.py --scene 0 --libs main steal --reps 8 > $O/ab_mesh_on.jsonl 2> $O/ab_mesh_on.err && cat $O/ab_mesh_on.jsonl &&
MCPT_STEAL=0 timeout -k 10 400 python tools/ab_interleave.py --scene 0 --libs main steal --reps 6 > $O/ab_mesh_off.jsonl 2> $O/ab_mesh_off.err && cat $O/ab_mesh_off.jsonl &&
MCPT_STEAL=1 timeout -k 10 400 python tools/ab_interleave.py --scene -1 --libs main steal --reps 6 > $O/ab_mesh4_on.jsonl 2> $O/ab_mesh4_on.err && cat $O/ab_mesh4_on.jsonl
