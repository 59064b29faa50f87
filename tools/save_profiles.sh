#!/bin/bash
# Copy one measurement session's results (tools/gpu_round_check.sh TAG) from gpurun_out/TAG into
# profiles/ under the round prefix:  tools/save_profiles.sh TAG [ROUND=r01]
set -e
V=$1; R=${2:-r01}; O=gpurun_out/$V; P=profiles/${R}_${V}
cp $O/bench.json ${P}_bench.json
[ -f $O/bench_gloo2.json ] && cp $O/bench_gloo2.json ${P}_bench_gloo2_rehearsal.json
cp $O/prof/run_kernel_stats.csv ${P}_kernel_stats.csv
python tools/trace_summary.py $O/prof/run_kernel_trace.csv \
  "$R $V: rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline" > ${P}_kernel_trace_summary.txt
mkdir -p ${P}_pmc
for k in fetch sqa sqb sqc write; do
  f=$(ls $O/pmc/$k/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && cp $f ${P}_pmc/$k.csv
done
cp $O/pmc_traffic.json ${P}_pmc/ && cp $O/pmc_traffic.json profiles/pmc_traffic.json
cp $O/pytest_gpu.log ${P}_pytest_gpu.log
for f in configs shard_balance launch_shape; do
  [ -f $O/$f.jsonl ] && grep '^{' $O/$f.jsonl > ${P}_$f.jsonl
done
ls ${P}_*
