#!/bin/bash
# Copy one measurement session's results (tools/gpu_check.sh TAG) from gpurun_out/TAG into
# profiles/ under the round prefix:  tools/save_profiles.sh TAG [ROUND=r02]
# (a session split in two calls: save the bench call; copy the other's pmc_records.json and
# pytest log by hand)
# The PMC records (keyed by libmcpt.so's sha256) become profiles/pmc_records.json, which
# bench.py's roofline reads.
set -e
V=$1; R=${2:-r03}; O=gpurun_out/$V; P=profiles/${R}_${V}
cp $O/bench.json ${P}_bench.json
[ -f $O/bench_c4.json ] && cp $O/bench_c4.json ${P}_bench_c4.json
[ -f $O/bench_mesh.json ] && cp $O/bench_mesh.json ${P}_bench_mesh.json
[ -f $O/bench_gloo8.json ] && grep '^{' $O/bench_gloo8.json > ${P}_bench_gloo8_rehearsal.json
[ -f $O/bench_gloo8_strong.json ] && grep '^{' $O/bench_gloo8_strong.json > ${P}_bench_gloo8_strong_rehearsal.json
[ -f $O/bench_gloo2.json ] && grep '^{' $O/bench_gloo2.json > ${P}_bench_gloo2_rehearsal.json
[ -f $O/bench_gloo4.json ] && grep '^{' $O/bench_gloo4.json > ${P}_bench_gloo4_rehearsal.json
[ -f $O/bench_c1.json ] && cp $O/bench_c1.json ${P}_bench_c1.json
[ -f $O/bench_c3.json ] && cp $O/bench_c3.json ${P}_bench_c3.json
[ -f $O/bench_c5.json ] && cp $O/bench_c5.json ${P}_bench_c5.json
[ -f $O/bench_gloo2_c4.json ] && grep '^{' $O/bench_gloo2_c4.json > ${P}_bench_gloo2_c4_rehearsal.json
[ -f $O/bench_nccl2_1gpu.err ] && cp $O/bench_nccl2_1gpu.err ${P}_bench_nccl2_on_1gpu_refused.txt
cp $O/prof/run_kernel_stats.csv ${P}_kernel_stats.csv
python tools/trace_summary.py $O/prof/run_kernel_trace.csv \
  "$R $V: rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline" > ${P}_kernel_trace_summary.txt
# (raw counter CSVs are not kept: since round 5 the records below carry every counter per launch)
[ -f $O/pmc_records.json ] && cp $O/pmc_records.json ${P}_pmc_records.json && cp $O/pmc_records.json profiles/pmc_records.json
[ -f $O/pytest_gpu.log ] && cp $O/pytest_gpu.log ${P}_pytest_gpu.log
for f in configs shard_balance launch_shape; do
  [ -f $O/$f.jsonl ] && grep '^{' $O/$f.jsonl > ${P}_$f.jsonl
done
ls ${P}_*
