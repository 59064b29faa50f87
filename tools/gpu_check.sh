#!/bin/bash
# One GPU-box session: parity tests, smoke, PMC passes of the C2 and C4 bench workloads
# (-> profiles/pmc_records.json records keyed by libmcpt.so's sha256, which bench.py's
# roofline reads), bench lines of every BASELINE config (C2, C4, C3 sweep, C5, C1), the
# kernel-trace profile, and (full) the N>1 rehearsals: plain `bench.py --gpus N` with gloo
# ranks sharing the one GPU (bench.py starts its own ranks).  Every GPU step has its own time
# limit; the chain stops at the first failure.
#   tools/gpu_check.sh TAG [notest] [nopmc] [pmcall] [nobench] [full]   (flags in any order)
set -o pipefail
has() { local f; for f in "${@:2}"; do [ "$f" = "$1" ] && return 0; done; return 1; }
FLAGS=("${@:2}")
export TMPDIR=/tmp
O=gpurun_out/${1:-run}
mkdir -p $O
if ! has notest "${FLAGS[@]}"; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 && echo "pytest ok" &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" || exit $?
fi
cp profiles/pmc_records.json $O/pmc_records.json 2>/dev/null
if ! has nopmc "${FLAGS[@]}"; then
  bash tools/pmc.sh $O/pmc && echo "pmc c2 ok" &&
  python tools/pmc_summary.py $O/pmc scene6_1920x1080_256spp_B8 $O/pmc_records.json > /dev/null &&
  bash tools/pmc.sh $O/pmc_c4 --config c4 && echo "pmc c4 ok" &&
  python tools/pmc_summary.py $O/pmc_c4 scene8_1920x1080_512spp_B12 $O/pmc_records.json > /dev/null &&
  PMC_MEM=1 bash tools/pmc.sh $O/pmc_mesh --config mesh && echo "pmc mesh ok" &&
  python tools/pmc_summary.py $O/pmc_mesh mesh1000k_1920x1080_64spp_B8 $O/pmc_records.json > /dev/null &&
  cp $O/pmc_records.json profiles/pmc_records.json || exit $?
fi
if has pmcall "${FLAGS[@]}"; then   # PMC records for the C3 line's dominant point, C5 and C1 too
  bash tools/pmc.sh $O/pmc_c3 --config c3 --rough 0 && echo "pmc c3 ok" &&
  python tools/pmc_summary.py $O/pmc_c3 scene6_1920x1080_1024spp_B8_ior1.5_rough0 $O/pmc_records.json > /dev/null &&
  bash tools/pmc.sh $O/pmc_c5 --config c5 && echo "pmc c5 ok" &&
  python tools/pmc_summary.py $O/pmc_c5 scene6_3840x2160_1024spp_B8 $O/pmc_records.json --launches=1 > /dev/null &&
  bash tools/pmc.sh $O/pmc_c1 --config c1 && echo "pmc c1 ok" &&
  python tools/pmc_summary.py $O/pmc_c1 scene1_256x256_4spp_B3 $O/pmc_records.json > /dev/null &&
  cp $O/pmc_records.json profiles/pmc_records.json || exit $?
fi
has nobench "${FLAGS[@]}" && exit 0
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && cat $O/bench.json &&
timeout -k 10 400 python bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err &&
echo "bench c4 ok" && cat $O/bench_c4.json &&
timeout -k 10 400 python bench.py --config mesh > $O/bench_mesh.json 2> $O/bench_mesh.err &&
echo "bench mesh ok" && cat $O/bench_mesh.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err && echo "prof ok" &&
timeout -k 10 200 python bench.py --config c1 > $O/bench_c1.json 2> $O/bench_c1.err && echo "bench c1 ok" &&
timeout -k 10 400 python bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err && echo "bench c3 ok" &&
timeout -k 10 400 python bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err && echo "bench c5 ok" || exit $?
has full "${FLAGS[@]}" || exit 0
# N>1 path rehearsal on the one GPU: the ranks share cuda:0 with gloo collectives (RCCL needs
# one GPU per rank; the driver runs the real N>1 nccl bench on an 8-GPU node)
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err && echo "gloo2 ok" &&
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo4.json 2> $O/bench_gloo4.err && echo "gloo4 ok" &&
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --config c4 \
  > $O/bench_gloo2_c4.json 2> $O/bench_gloo2_c4.err && echo "gloo2 c4 ok" &&
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo8.json 2> $O/bench_gloo8.err && echo "gloo8 ok" &&
MCPT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline --scaling strong \
  > $O/bench_gloo8_strong.json 2> $O/bench_gloo8_strong.err && echo "gloo8 strong ok" &&
{ timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_nccl2_1gpu.json \
    2> $O/bench_nccl2_1gpu.err; rc=$?; echo "nccl2 on one GPU: exit $rc (expected non-zero, no line)";
  [ $rc -ne 0 ] && [ ! -s $O/bench_nccl2_1gpu.json ]; }
