#!/bin/bash
# One GPU-box session: GPU parity suite, row-partition shard balance (balanced vs bands), and
# the all-configs measurement.  tools/gpu_partition_check.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-partition}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python tools/shard_balance.py --bands 8 > $O/shard_balance.jsonl 2> $O/shard.err &&
echo "shards ok" &&
timeout -k 10 500 python tools/configs_bench.py > $O/configs.jsonl 2> $O/configs.err && echo "configs ok"
