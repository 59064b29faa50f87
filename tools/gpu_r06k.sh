# round 6 session k: the 1/8-frame C2 launch (strong scaling at N = 8): occupancy over time and segments per item
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06k}; mkdir -p $O
BT=$PWD/montecarlo-pathtracing_amd/mcpt/variants/libmcpt_blocktimes.so
MCPT_LIB=$BT timeout -k 10 200 python tools/blocktimes.py c2 --auto --shard 8 > $O/bt_c2_shard8.jsonl 2>&1 &&
MCPT_LIB=$BT timeout -k 10 200 python tools/blocktimes.py c2 --auto > $O/bt_c2_full.jsonl 2>&1 &&
for k in 1 2 4; do MCPT_SEG_PER_ITEM=$k timeout -k 10 200 python tools/strong_scaling_projection.py --worlds 8 > $O/strong8_seg$k.jsonl 2>&1 || exit 1; done
MCPT_PASS_SPLIT=1 timeout -k 10 200 python tools/strong_scaling_projection.py --worlds 8 > $O/strong8_passsplit.jsonl 2>&1
cat $O/bt_c2_shard8.jsonl $O/bt_c2_full.jsonl; for f in $O/strong8_*.jsonl; do echo $f; grep -o '"projected_step_ms": [0-9.]*' $f; done
