#!/bin/bash
# gemm8n bring-up: numerics tests, then per-shape A/B (DTC_GEMM8N=0 vs 3), then whole-step A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_n8_gpu.py > gpurun_out/n8_tests.log 2>&1; rc=$?
tail -n 15 gpurun_out/n8_tests.log
[ $rc -ne 0 ] && exit $rc
DTC_GEMM8N=0 timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --no-ref > gpurun_out/n8_bench0.log 2>&1 || exit $?
DTC_GEMM8N=3 timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 > gpurun_out/n8_bench3.log 2>&1 || exit $?
paste gpurun_out/n8_bench0.log gpurun_out/n8_bench3.log | head -40
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM8N=0" "DTC_GEMM8N=3" "DTC_GEMM8N=1"
