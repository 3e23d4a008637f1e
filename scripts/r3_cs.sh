#!/bin/bash
# fused wgrad bias sums: tests (wgrad, kernels), whole-step A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_n8_gpu.py tests/test_kernels_gpu.py > gpurun_out/cs_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/cs_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_WGRAD_CS256=0" "DTC_WGRAD_CS256=1"
