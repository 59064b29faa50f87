# round 6 session e: mesh layout variants B2 / D / D2 against round 5's layout
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06e}; mkdir -p $O
MCPT_LIB=$PWD/montecarlo-pathtracing_amd/mcpt/variants/libmcpt_meshD2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_meshes.py tests/test_gpu_queries.py tests/test_gpu_full_size.py -k "mesh or Mesh or trace or hit" -x -q --timeout 300 --timeout-method thread > $O/pytest_meshD2.log 2>&1; rc=$?; echo "pytest D2 rc=$rc"; tail -3 $O/pytest_meshD2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_interleave.py --scene 0 --libs meshD meshD2 meshB2 r05mesh --reps 8 > $O/ab_mesh.jsonl 2> $O/ab_mesh.err && cat $O/ab_mesh.jsonl &&
timeout -k 10 300 python tools/ab_interleave.py --scene -1 --libs meshD meshD2 meshB2 r05mesh --reps 6 > $O/ab_mesh4.jsonl 2> $O/ab_mesh4.err && cat $O/ab_mesh4.jsonl
