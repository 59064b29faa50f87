# round 6 session d: mesh layout variants (B: both leaf triangles in the node step; C: one shared
# triangle block per step) against round 5's layout, and C's bits
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06d}; mkdir -p $O
MCPT_LIB=$PWD/montecarlo-pathtracing_amd/mcpt/variants/libmcpt_meshC.so timeout -k 10 900 python -u -m pytest tests/test_gpu_meshes.py tests/test_gpu_queries.py tests/test_gpu_full_size.py -k "mesh or Mesh or trace or hit" -x -q --timeout 300 --timeout-method thread > $O/pytest_meshC.log 2>&1; rc=$?; echo "pytest C rc=$rc"; tail -3 $O/pytest_meshC.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_interleave.py --scene 0 --libs meshC meshB r05mesh --reps 8 > $O/ab_mesh.jsonl 2> $O/ab_mesh.err && cat $O/ab_mesh.jsonl &&
timeout -k 10 300 python tools/ab_interleave.py --scene -1 --libs meshC meshB r05mesh --reps 6 > $O/ab_mesh4.jsonl 2> $O/ab_mesh4.err && cat $O/ab_mesh4.jsonl
