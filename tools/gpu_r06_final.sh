#!/bin/bash
# Round-6 measurement session on one GPU box, in parts (each GPU step under its own limit, the
# chain stops at the first failure):
#   tools/gpu_r06_final.sh TAG tests   — the GPU suite and smoke()
#   tools/gpu_r06_final.sh TAG pmc     — PMC passes of every bench workload -> pmc_records.json (same build)
#   tools/gpu_r06_final.sh TAG bench   — bench lines of every config, the rocprofv3 kernel trace, C5 to 84,000 spp
#   tools/gpu_r06_final.sh TAG dist    — N > 1 rehearsals (gloo ranks sharing the GPU): default (strong) and weak
#   tools/gpu_r06_final.sh TAG pmc2    — the C2 record again, averaged over 6 timed calls
#   tools/gpu_r06_final.sh TAG c5full  — tools/c5_full.py alone
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
case "$2" in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" ;;
pmc)   # each record averages the last 4 timed calls' launches (PMC_STEPS, --calls)
  cp profiles/pmc_records.json $O/pmc_records.json
  export PMC_STEPS=4
  for spec in "c2 scene6_1920x1080_256spp_B8" "c4 scene8_1920x1080_512spp_B12" "c1 scene1_256x256_4spp_B3"; do
    set -- $spec
    bash tools/pmc.sh $O/pmc_$1 --config $1 && python tools/pmc_summary.py $O/pmc_$1 $2 $O/pmc_records.json --calls=4 > /dev/null && echo "pmc $1 ok" || exit 1
  done
  bash tools/pmc.sh $O/pmc_c3 --config c3 --rough 0 && python tools/pmc_summary.py $O/pmc_c3 scene6_1920x1080_1024spp_B8_ior1.5_rough0 $O/pmc_records.json --calls=4 > /dev/null && echo "pmc c3 ok" &&
  bash tools/pmc.sh $O/pmc_c5 --config c5 && python tools/pmc_summary.py $O/pmc_c5 scene6_3840x2160_1024spp_B8 $O/pmc_records.json --launches=1 --calls=4 > /dev/null && echo "pmc c5 ok" &&
  PMC_MEM=1 bash tools/pmc.sh $O/pmc_mesh --config mesh && python tools/pmc_summary.py $O/pmc_mesh mesh1000k_1920x1080_64spp_B8 $O/pmc_records.json --calls=4 > /dev/null && echo "pmc mesh ok" &&
  PMC_MEM=1 bash tools/pmc.sh $O/pmc_mesh_big --config mesh_big && python tools/pmc_summary.py $O/pmc_mesh_big mesh4x1000k_1920x1080_64spp_B8 $O/pmc_records.json --calls=4 > /dev/null && echo "pmc mesh_big ok" ;;
bench)
  for c in c2 c4 mesh mesh_big c1 c3 c5; do
    timeout -k 10 600 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err && echo "bench $c ok: $(python -c "import json;d=json.load(open('$O/bench_$c.json'));print(d['value'], d['roofline'].get('frac'))")" || exit 1
  done
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err && echo "prof ok" &&
  timeout -k 10 400 python tools/c5_full.py > $O/c5_full.jsonl 2> $O/c5_full.err && echo "c5 full ok" && tail -1 $O/c5_full.jsonl ;;
dist)
  MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_gloo2.json 2> $O/bench_gloo2.err && echo "gloo2 ok" &&
  MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_gloo4.json 2> $O/bench_gloo4.err && echo "gloo4 ok" &&
  MCPT_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_gloo8_strong.json 2> $O/bench_gloo8_strong.err && echo "gloo8 strong ok" &&
  MCPT_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline --scaling weak > $O/bench_gloo8_weak.json 2> $O/bench_gloo8_weak.err && echo "gloo8 weak ok" &&
  MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --config c4 > $O/bench_gloo2_c4.json 2> $O/bench_gloo2_c4.err && echo "gloo2 c4 ok" &&
  MCPT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_gloo2_torchrun.json 2> $O/bench_gloo2_torchrun.err && echo "gloo2 torchrun ok" ;;
pmc2)   # the headline's record again: every counter pass on one schedule (lane walk, PMC_SEG segments
  # per item, default 4: AUTO settles on 4, or on 2 in some runs — r06x, r06q), 4 timed calls
  # averaged; records of other schedules stay beside it (pmc_summary.merge_record)
  cp profiles/pmc_records.json $O/pmc_records.json
  MCPT_SEG_PER_ITEM=${PMC_SEG:-4} PMC_STEPS=4 bash tools/pmc.sh $O/pmc_c2 && python tools/pmc_summary.py $O/pmc_c2 scene6_1920x1080_256spp_B8 $O/pmc_records.json --calls=4 > $O/pmc_c2_summary.json && echo "pmc c2 ok" ;;
c5full)
  timeout -k 10 400 python tools/c5_full.py > $O/c5_full.jsonl 2> $O/c5_full.err && echo "c5 full ok" && head -1 $O/c5_full.jsonl && tail -1 $O/c5_full.jsonl ;;
esac
