#!/bin/bash
# round 6 session n: the mesh-space ray of the walk in LDS (MCPT_MRAY=1/2) and the mesh scene unstaged
# (MCPT_MESH_NO_LDS) and 32-bit record offsets (MCPT_REC32), interleaved against the shipped library on both mesh workloads
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06n}; mkdir -p $O
timeout -k 10 400 python tools/ab_interleave.py --scene 0 --libs main mr1 mr1n mr0n mr2 ro ro_mr1 ro_mr1n --reps 8 > $O/ab_mesh.jsonl 2> $O/ab_mesh.err && cat $O/ab_mesh.jsonl &&
timeout -k 10 400 python tools/ab_interleave.py --scene -1 --libs main mr1 mr1n mr0n mr2 ro ro_mr1 ro_mr1n --reps 6 > $O/ab_mesh4.jsonl 2> $O/ab_mesh4.err && cat $O/ab_mesh4.jsonl
