#!/bin/bash
# round 6 session p: the mesh pair record's range flag for rcp6_rn and the scalar suspension compare
# (rf) against main (t13 of session o): parity on the mesh tests, interleaved timing, walk exit
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06p}; mkdir -p $O
MCPT_LIB=$PWD/montecarlo-pathtracing_amd/mcpt/variants/libmcpt_rf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_meshes.py tests/test_gpu_full_size.py tests/test_gpu_stream.py -k "mesh or Mesh" -x -q --timeout 300 --timeout-method thread > $O/pytest_rf.log 2>&1; rc=$?; echo "pytest rf rc=$rc"; tail -3 $O/pytest_rf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_interleave.py --scene 0 --libs main rf --walk-exit 16 24 32 --reps 8 > $O/ab_mesh.jsonl 2> $O/ab_mesh.err && cat $O/ab_mesh.jsonl &&
timeout -k 10 400 python tools/ab_interleave.py --scene -1 --libs main rf --walk-exit 24 32 --reps 6 > $O/ab_mesh4.jsonl 2> $O/ab_mesh4.err && cat $O/ab_mesh4.jsonl
