#!/bin/bash
MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_trk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/trk_pytest.log 2>&1 || exit 1
bash tools/gpu_libs_ab.sh r02p "6 8 3 5" 256 "2 4" main trk bias
