#!/bin/bash
# whole-step A/B of the phase-interleaved 256^2 main loop (GPT-2 small, 1 GPU)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_sk_gpu.py -m gpu -k "gemm or lmhead or ce_ or sk" > gpurun_out/r3_g8ps_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/r3_g8ps_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM8P=1" "DTC_GEMM8P=0"
