#!/bin/bash
bash tools/gpu_bench3.sh r02r && bash tools/gpu_libs_ab.sh r02r "6 8 3 5 1" 256 "2 4" main prev
