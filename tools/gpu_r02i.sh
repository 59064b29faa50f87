export TMPDIR=/tmp; O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 400 python tools/configs_bench.py > $O/configs.jsonl 2> $O/configs.err && echo configs ok &&
timeout -k 10 300 python tools/c5_full.py --traversal 1 --seg-per-item 2 > $O/c5_full.jsonl 2> $O/c5.err && echo c5 ok &&
timeout -k 10 120 ./montecarlo-pathtracing_amd/bin/mcpt_render --scene 8 --width 1920 --height 1080 --spp 512 --bounces 12 --chunk 512 --devices 0,0,0,0,0,0,0,0 > $O/app_c4_8shards.json 2>&1 &&
timeout -k 10 120 ./montecarlo-pathtracing_amd/bin/mcpt_render --scene 8 --width 1920 --height 1080 --spp 512 --bounces 12 --chunk 512 > $O/app_c4_1.json 2>&1 && echo app ok &&
bash tools/gpu_libs_ab.sh r02i "8 3 7" 256 "1 4" main l2w8
