#!/bin/bash
# stream-K GEMM: numerics + determinism, then GPT-2 small layer shapes with and without it
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gemm_sk_gpu.py -m gpu > gpurun_out/r3_sk_tests.log 2>&1; rc=$?
echo "sk tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/r3_sk_tests.log | head -30
[ $rc -ne 0 ] && exit $rc
for v in 0 3; do
  DTC_GEMM_SK=$v timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --only "fwd ,dgrad" --no-ref > gpurun_out/r3_sk_bench_$v.log 2>&1 || exit $?
  echo "== DTC_GEMM_SK=$v"; grep -v amdgpu.ids gpurun_out/r3_sk_bench_$v.log
done
