#!/bin/bash
# Full measurement session on one GPU box: tools/gpu_check.sh (parity suite, smoke, PMC passes,
# bench, rocprof kernel trace, N=2 gloo rehearsal), then all BASELINE configs, 8-GPU shard
# balance of both row partitions, and launch-shape costs.  tools/gpu_round_check.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
bash tools/gpu_check.sh $1 full &&
timeout -k 10 500 python tools/configs_bench.py > $O/configs.jsonl 2> $O/configs.err && echo "configs ok" &&
timeout -k 10 300 python tools/shard_balance.py --bands 8 > $O/shard_balance.jsonl 2> $O/shard.err &&
echo "shards ok" &&
timeout -k 10 300 python tools/launch_shape_cost.py > $O/launch_shape.jsonl 2> $O/shape.err && echo "shape ok"
