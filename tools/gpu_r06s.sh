#!/bin/bash
# round 6 session s: the mesh kernel's scene-node box tests without exec-mask branches (T4) against main
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06s}; mkdir -p $O
timeout -k 10 400 python tools/ab_interleave.py --scene 0 --libs main t4 --reps 10 > $O/ab_mesh.jsonl 2> $O/ab_mesh.err && cat $O/ab_mesh.jsonl &&
timeout -k 10 400 python tools/ab_interleave.py --scene -1 --libs main t4 --reps 8 > $O/ab_mesh4.jsonl 2> $O/ab_mesh4.err && cat $O/ab_mesh4.jsonl
