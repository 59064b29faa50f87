#!/bin/bash
bash tools/gpu_libs_ab.sh r02v "6 8 3 1" 256 "2 4" main slp
