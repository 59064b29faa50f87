#!/bin/bash
bash tools/gpu_bench3.sh r02q && bash tools/gpu_libs_ab.sh r02q "6 8 3 5 1" 256 "2 4" main dcull fc_l2f3 fc_l2f5
