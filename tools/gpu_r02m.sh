#!/bin/bash
bash tools/gpu_libs_ab.sh r02m "6 1 2 4 8" 256 "2" main wfm w8 && bash tools/gpu_libs_ab.sh r02m2 "6" 256 "2" wfm main w8
