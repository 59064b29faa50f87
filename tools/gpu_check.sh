#!/bin/bash
# One GPU-box session: parity tests, smoke, PMC passes (-> profiles/pmc_traffic.json for the
# bench's `traffic`/`valu` fields), bench, kernel-trace profile, and (full) the N=2 gloo
# rehearsal.  Every GPU step has its own time limit; the chain stops at the first failure.
#   tools/gpu_check.sh TAG [full]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-run}
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
bash tools/pmc.sh $O/pmc && echo "pmc ok" &&
python tools/pmc_summary.py $O/pmc scene6_1920x1080_256spp_B8 $O/pmc_traffic.json > /dev/null &&
cp $O/pmc_traffic.json profiles/pmc_traffic.json &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && cat $O/bench.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err && echo "prof ok" || exit $?
[ "${2:-}" = "full" ] || exit 0
# N>1 path rehearsal on the one GPU: 2 ranks share cuda:0, gloo collectives (RCCL needs
# one GPU per rank; the driver runs the real N>1 nccl bench on an 8-GPU node)
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err && echo "gloo2 ok" && cat $O/bench_gloo2.json
