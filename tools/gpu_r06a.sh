set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_checked.py -x -v --timeout 300 --timeout-method thread > $O/pytest_checked.log 2>&1; echo "pytest checked rc=$?"
tail -5 $O/pytest_checked.log
MCPT_SEG_PER_ITEM=4 timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 2 > $O/b_c5_4.json 2> $O/b_c5_4.err && echo "c5 K4 ok" && cat $O/b_c5_4.json | head -c 400 &&
MCPT_LIB=$PWD/montecarlo-pathtracing_amd/mcpt/variants/libmcpt_checked.so MCPT_SEG_PER_ITEM=4 timeout -k 10 400 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > $O/b_c5_4_checked.json 2> $O/b_c5_4_checked.err && echo "c5 K4 checked ok"
