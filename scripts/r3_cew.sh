#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "ce_ or lmhead or p2p" > gpurun_out/r3_cew_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r3_cew_tests.log | tail -n 2
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_dist_gpu.py -m gpu > gpurun_out/r3_cew_engine.log 2>&1; rc=$?
echo "engine rc=$rc"; tail -n 2 gpurun_out/r3_cew_engine.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_CE_WGRAD=1" "DTC_CE_WGRAD=0" "DTC_CE_WGRAD=1|--model ref" "DTC_CE_WGRAD=0|--model ref"
