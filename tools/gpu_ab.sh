#!/bin/bash
# Kernel A/B harness (one GPU box session): timing of candidate builds/settings of the render
# kernel, interleaved so that every candidate sees the same box state, optionally preceded by
# the parity suites on each candidate.  Replaces round 1-2's one-off session scripts
# (gpu_libs_ab.sh, ab_libs.sh, gpu_env_ab.sh, gpu_lib_env_ab.sh, gpu_env_spp_ab.sh,
# gpu_variant_ab.sh, gpu_rr_ab.sh, gpu_r02*.sh, ...; profiles/README.md maps each committed
# A/B file to the invocation that reproduces it).
#
#   tools/gpu_ab.sh TAG [options] CAND...
#     CAND     = LIB[@VAR=VALUE[@VAR=VALUE...]]
#                LIB "main" = the in-tree libmcpt.so, else variants/libmcpt_<LIB>.so;
#                each VAR=VALUE is exported for that candidate only (e.g. main@MCPT_LEAF_BATCH=4)
#     --scenes "6 8"  scenes (default "6 8")
#     --spp N         passes per timed launch (default 256)
#     --reps R        timed launches per (candidate, K, scene) (default 3)
#     --k "1 2 4"     pass segments per work item (MCPT_SEG_PER_ITEM), interleaving loop (default "2")
#     --modes "1"     traversal modes (1 per-lane, 2 wave-coherent, 3 stream; default "1")
#     --walk-exit "16 32"  per-lane walks' suspension thresholds to time (default: the library's)
#     --parity        run the parity suites (tests/test_gpu_parity.py, test_gpu_paths.py) on every
#                     candidate first; stop at the first failure
#     --stamps        also run tools/stamps.py with the stamps variant library (diagnostic build)
# Output: gpurun_out/TAG/ab.jsonl (one line per candidate x K x scene x mode), pytest logs.
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
SCENES="6 8"; SPP=256; REPS=3; KS="2"; MODES="1"; PARITY=0; STAMPS=0; WX="-1"
while [ $# -gt 0 ]; do
  case "$1" in
    --scenes) SCENES=$2; shift 2 ;;
    --spp) SPP=$2; shift 2 ;;
    --reps) REPS=$2; shift 2 ;;
    --k) KS=$2; shift 2 ;;
    --modes) MODES=$2; shift 2 ;;
    --walk-exit) WX=$2; shift 2 ;;
    --parity) PARITY=1; shift ;;
    --stamps) STAMPS=1; shift ;;
    *) break ;;
  esac
done
[ $# -gt 0 ] || { echo "usage: tools/gpu_ab.sh TAG [options] CAND..."; exit 2; }
O=gpurun_out/$TAG; mkdir -p $O
V=montecarlo-pathtracing_amd/mcpt

libpath() { if [ "$1" = main ]; then echo $V/libmcpt.so; else echo $V/variants/libmcpt_$1.so; fi; }

# run CMD... with candidate $1's library and environment (in a subshell)
with_cand() {
  local cand=$1; shift
  ( IFS=@ read -r lib settings <<< "$cand"
    export MCPT_LIB=$(libpath "$lib")
    [ -f "$MCPT_LIB" ] || { echo "missing $MCPT_LIB"; exit 2; }
    IFS=@; for s in $settings; do export "$s"; done; unset IFS
    "$@" )
}

if [ $PARITY = 1 ]; then
  for c in "$@"; do
    n=$(echo "$c" | tr '@=/' '___')
    with_cand "$c" timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q \
      --timeout 300 --timeout-method thread > $O/pytest_$n.log 2>&1 ||
      { echo "parity FAILED for $c"; tail -20 $O/pytest_$n.log; exit 1; }
    echo "parity ok: $c ($(tail -1 $O/pytest_$n.log))"
  done
fi
for k in $KS; do
  for c in "$@"; do
    with_cand "$c" env MCPT_SEG_PER_ITEM=$k timeout -k 10 300 python tools/ab_time.py --scenes $SCENES \
      --modes $MODES --spp $SPP --reps $REPS --walk-exit $WX --tag "${c}_K$k" >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  done
done
cat $O/ab.jsonl
if [ $STAMPS = 1 ]; then
  MCPT_LIB=$V/variants/libmcpt_stamps.so timeout -k 10 200 python tools/stamps.py > $O/stamps.jsonl 2>&1 &&
    grep '^{' $O/stamps.jsonl
fi
