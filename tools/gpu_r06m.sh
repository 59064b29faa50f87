# round 6 session m: render lanes on C5 / C4 shard / C2 shard 4, and C2's segments per item with lanes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06m}; mkdir -p $O
timeout -k 10 600 python tools/lanes_ab.py --cases c5 c4_shard8 c2_shard4 --calls 6 > $O/lanes_ab2.jsonl 2> $O/lanes_ab2.err || exit 1
for k in 1 2 4; do MCPT_SEG_PER_ITEM=$k timeout -k 10 300 python tools/lanes_ab.py --cases c2 c2_shard8 > $O/lanes_seg$k.jsonl 2> $O/lanes_seg$k.err || exit 1; done
for f in $O/lanes_ab2.jsonl $O/lanes_seg*.jsonl; do echo $f; python -c "
import sys,json
for l in open('$f'):
  d=json.loads(l); print(d['case'], d['schedule']['seg_per_item'], d['median_lanes'], d['median_in_order'], d['gain'], d['bit_equal'])"; done
