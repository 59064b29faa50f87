#!/bin/bash
# C1 bench line + the N>1 path rehearsed on one GPU (2 and 4 ranks share cuda:0, gloo
# collectives; every rank-0 line carries the gathered frame's self check):
#   tools/gpu_rehearse.sh TAG
export TMPDIR=/tmp; O=gpurun_out/${1:-rehearse}; mkdir -p $O
timeout -k 10 200 python bench.py --config c1 > $O/bench_c1.json 2> $O/bench_c1.err && echo "bench c1 ok" &&
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err && echo "gloo2 ok" &&
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo4.json 2> $O/bench_gloo4.err && echo "gloo4 ok" &&
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --config c4 \
  > $O/bench_gloo2_c4.json 2> $O/bench_gloo2_c4.err && echo "gloo2 c4 ok"
