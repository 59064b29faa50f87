# round 6 session c: mesh record layout (last-level records with both leaf triangles): mesh tests, A/B vs round 5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_meshes.py tests/test_gpu_queries.py tests/test_gpu_full_size.py -k "mesh or Mesh or trace or hit" -x -q --timeout 300 --timeout-method thread > $O/pytest_mesh.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_mesh.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_interleave.py --scene 0 --libs main r05mesh --reps 8 > $O/ab_mesh.jsonl 2> $O/ab_mesh.err && cat $O/ab_mesh.jsonl &&
timeout -k 10 300 python tools/ab_interleave.py --scene -1 --libs main r05mesh --reps 6 > $O/ab_mesh4.jsonl 2> $O/ab_mesh4.err && cat $O/ab_mesh4.jsonl
