# round 6 session l: render lanes — bits, gain on the bench workloads, projected strong scaling
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06l}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "render_lanes or tail_pieces or item_order" -x -q --timeout 300 --timeout-method thread > $O/pytest_lanes.log 2>&1; rc=$?; tail -3 $O/pytest_lanes.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/lanes_ab.py --cases c2 c2_shard8 c4 mesh > $O/lanes_ab.jsonl 2> $O/lanes_ab.err; rc=$?; cat $O/lanes_ab.jsonl | python -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['case'], d['median_lanes'], d['median_in_order'], d['gain'], d['bit_equal'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/strong_scaling_projection.py > $O/strong_c2.jsonl 2>&1 && grep -o '"world": [0-9]*\|"projected_step_ms": [0-9.]*\|"efficiency": [0-9.]*' $O/strong_c2.jsonl
