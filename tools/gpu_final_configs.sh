#!/bin/bash
# final config sweep + C5 at its full target + C++ host N-shard run
export TMPDIR=/tmp; O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 400 python tools/configs_bench.py > $O/configs.jsonl 2> $O/configs.err && echo configs ok &&
timeout -k 10 300 python tools/c5_full.py --traversal 1 --seg-per-item 2 > $O/c5_full.jsonl 2> $O/c5.err && echo c5 ok &&
timeout -k 10 120 ./montecarlo-pathtracing_amd/bin/mcpt_render --scene 6 --width 1920 --height 1080 --spp 256 --bounces 8 --chunk 256 --devices 0,0,0,0,0,0,0,0 > $O/app_c2_8shards.json 2>&1 &&
timeout -k 10 120 ./montecarlo-pathtracing_amd/bin/mcpt_render --scene 6 --width 1920 --height 1080 --spp 256 --bounces 8 --chunk 256 > $O/app_c2_1.json 2>&1 && echo app ok
