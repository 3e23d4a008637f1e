#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "attention" > gpurun_out/r3_attn_tests.log 2>&1; rc=$?
echo "attn tests rc=$rc"; tail -n 2 gpurun_out/r3_attn_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for qg in 1 2; do
  DTC_ATTN_QG=$qg timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 > gpurun_out/r3_attn_qg$qg.log 2>&1 || exit $?
  echo "QG=$qg: $(grep attn gpurun_out/r3_attn_qg$qg.log | tr '\n' ' ')"
done
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_ATTN_QG=2" "DTC_ATTN_QG=1"
