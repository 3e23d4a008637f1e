#!/bin/bash
# gemm8n with the overlapped epilogue: tests, per-shape (mask 3 vs 7), whole-step A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_n8_gpu.py > gpurun_out/n8_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/n8_tests.log
[ $rc -ne 0 ] && exit $rc
for m in 3 7; do
  DTC_GEMM8N=$m timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --no-ref --only qkv,out,fc1,fc2 > gpurun_out/n8_bench$m.log 2>&1 || exit $?
done
paste gpurun_out/n8_bench3.log gpurun_out/n8_bench7.log | cut -c1-150
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM8N=3" "DTC_GEMM8N=7"
