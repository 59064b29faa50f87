#!/bin/bash
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/paths592.log 2>&1; rc=$?; tail -2 gpurun_out/paths592.log; exit $rc
