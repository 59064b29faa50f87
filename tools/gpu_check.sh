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
[ "${2:-}" = "full" ] || exit 0
# N>1 path rehearsal on the one GPU: 2 ranks share cuda:0, gloo collectives (RCCL needs
# one GPU per rank; the driver runs the real N>1 nccl bench on an 8-GPU node)
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err && echo "gloo2 ok" && cat $O/bench_gloo2.json &&
bash tools/pmc.sh $O/pmc && echo "pmc ok"
