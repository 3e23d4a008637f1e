#!/bin/bash
# phase-interleaved 256^2 GEMM (gemm8p_kernel): numerics, then per-shape A/B vs gemm256_kernel
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or lmhead or ce_" > gpurun_out/r3_g8p_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 gpurun_out/r3_g8p_tests.log
[ $rc -ne 0 ] && exit $rc
for v in "DTC_GEMM8P=0" "DTC_GEMM8P=1" "DTC_GEMM8P=1 DTC_BIG_MIN_TILES=128"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 > gpurun_out/r3_g8p_bench_$tag.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r3_g8p_bench_$tag.log
done
