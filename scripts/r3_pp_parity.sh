#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py -m gpu > gpurun_out/r3_dist_gpu.log 2>&1; rc=$?
echo "dist rc=$rc"; tail -n 4 gpurun_out/r3_dist_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/parity_runs.sh
