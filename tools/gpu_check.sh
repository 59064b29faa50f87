#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile.  Every GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-run}
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && cat $O/bench.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err && echo "prof ok"
