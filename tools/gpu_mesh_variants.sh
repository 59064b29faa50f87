#!/bin/bash
# GPU session: mesh parity + large-mesh throughput for variant libraries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for v in "$@"; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$v.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_meshes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 \
    || { echo "variant $v parity FAILED"; tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$v.so timeout -k 10 600 python -u tools/big_mesh_bench.py \
    --sizes 10000 1000000 --spp 16 > $O/bm_$v.jsonl 2> $O/bm_$v.err || exit $?
  python -c "
import json,sys
for l in open('$O/bm_$v.jsonl'):
    d=json.loads(l); print('$v', d['triangles_per_instance'], d['traversal'], d['msamples_s'])"
done
