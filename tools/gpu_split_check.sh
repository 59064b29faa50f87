#!/bin/bash
# GPU session: full GPU test suite, then BASELINE C5 at its full 84,000-spp target per shard.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-split}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest ok" && tail -2 $O/pytest_gpu.log &&
timeout -k 10 400 python -u tools/c5_full.py > $O/c5_full.jsonl 2> $O/c5_full.err && echo "c5 ok" && cat $O/c5_full.jsonl
