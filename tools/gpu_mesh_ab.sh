#!/bin/bash
# mesh-kernel A/B: parity of the variants on the mesh tests, then big-mesh and small-mesh timing
#   tools/gpu_mesh_ab.sh OUTTAG lib1 lib2 ...   (lib "main" = in-tree libmcpt.so)
export TMPDIR=/tmp; O=gpurun_out/$1; shift; mkdir -p $O
for w in "$@"; do
  if [ "$w" = main ]; then L=montecarlo-pathtracing_amd/mcpt/libmcpt.so; else L=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$w.so; fi
  MCPT_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_meshes.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$w.log 2>&1 || { echo "$w mesh parity FAILED"; tail -5 $O/pytest_$w.log; exit 1; }
  MCPT_LIB=$L timeout -k 10 300 python tools/big_mesh_bench.py --sizes 10000 100000 1000000 --spp 32 > $O/big_$w.jsonl 2>> $O/err.log || exit 1
done
for w in "$@"; do python3 -c "
import json,sys
for l in open('$O/big_$w.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$w', d['triangles_per_instance'], d['traversal'], d['msamples_s'])"; done
