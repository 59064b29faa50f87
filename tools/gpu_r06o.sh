#!/bin/bash
# round 6 session o: the mesh walk's suspend test at the loop head (T1) and the mesh entry's set-up in
# a wave-uniform block with selects (T3), on the 32-bit record offsets (main): parity of T1+T3 on the
# mesh tests, then interleaved timing on both mesh workloads
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06o}; mkdir -p $O
MCPT_LIB=$PWD/montecarlo-pathtracing_amd/mcpt/variants/libmcpt_t13.so timeout -k 10 600 python -u -m pytest tests/test_gpu_meshes.py tests/test_gpu_full_size.py -k "mesh or Mesh" -x -q --timeout 300 --timeout-method thread > $O/pytest_t13.log 2>&1; rc=$?; echo "pytest t13 rc=$rc"; tail -3 $O/pytest_t13.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_interleave.py --scene 0 --libs main t1 t3 t13 --reps 10 > $O/ab_mesh.jsonl 2> $O/ab_mesh.err && cat $O/ab_mesh.jsonl &&
timeout -k 10 400 python tools/ab_interleave.py --scene -1 --libs main t1 t3 t13 --reps 8 > $O/ab_mesh4.jsonl 2> $O/ab_mesh4.err && cat $O/ab_mesh4.jsonl
