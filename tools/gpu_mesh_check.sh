#!/bin/bash
# GPU session: full GPU suite, then the large-mesh throughput table (tools/big_mesh_bench.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-mesh}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/big_mesh_bench.py ${2:-} > $O/big_mesh.jsonl 2> $O/big_mesh.err && cut -c1-260 $O/big_mesh.jsonl
timeout -k 10 300 python -u tools/mesh_bench.py > $O/mesh_scene.jsonl 2> $O/mesh_scene.err && cut -c1-300 $O/mesh_scene.jsonl
