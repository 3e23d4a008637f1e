#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "ce_ or lmhead" > gpurun_out/r3_cecs_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/r3_cecs_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3_cecs_bench.log 2>&1; rc=$?
tail -n 1 gpurun_out/r3_cecs_bench.log; exit $rc
