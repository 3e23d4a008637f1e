#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_n8_gpu.py -k "256x192 or forward or dgrad" > gpurun_out/p83_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/p83_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  DTC_GEMM8P3=$v timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --no-ref --only fc1,fc2 > gpurun_out/p83_bench$v.log 2>&1 || exit $?
done
paste gpurun_out/p83_bench0.log gpurun_out/p83_bench1.log | cut -c1-150
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM8P3=0" "DTC_GEMM8P3=1"
