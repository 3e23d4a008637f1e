#!/bin/bash
# 4-wave layer GEMM: tests, per-shape (4w off/on), whole-step A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_n8_gpu.py > gpurun_out/n8_tests.log 2>&1; rc=$?
tail -n 5 gpurun_out/n8_tests.log
[ $rc -ne 0 ] && exit $rc
for w in 0 1; do
  DTC_GEMM4W=$w DTC_GEMM8N=7 timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --no-ref --only qkv,out,fc1,fc2 > gpurun_out/w4_bench$w.log 2>&1 || exit $?
done
paste gpurun_out/w4_bench0.log gpurun_out/w4_bench1.log | cut -c1-150
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM4W=0" "DTC_GEMM4W=1" "DTC_GEMM4W=1 DTC_GEMM8N=7"
