#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or lmhead or ce_" > gpurun_out/r3_g8pc_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/r3_g8pc_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  DTC_GEMM8P=$v timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --only lm_head --no-ref > gpurun_out/r3_g8pc_bench_$v.log 2>&1 || exit $?
  echo "== DTC_GEMM8P=$v"; grep -v amdgpu.ids gpurun_out/r3_g8pc_bench_$v.log
done
