#!/bin/bash
bash tools/gpu_libs_ab.sh r02t "6 1 2 4" 256 "2 3" main w6
