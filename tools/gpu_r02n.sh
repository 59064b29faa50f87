#!/bin/bash
bash tools/gpu_bench3.sh r02n && bash tools/gpu_libs_ab.sh r02n "6 1 2 4 5 8" 256 "2" main prev
