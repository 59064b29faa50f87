#!/bin/bash
bash tools/gpu_libs_ab.sh r02o "8 3 5 7" 256 "2 4" main l2f1 l2f4 l2f5
