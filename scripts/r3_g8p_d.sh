#!/bin/bash
# asm transpose reads (no per-phase vmcnt(0)): numerics, lm_head + layer shapes incl. stream-K
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_sk_gpu.py -m gpu -k "gemm or lmhead or ce_ or sk" > gpurun_out/r3_g8pd_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/r3_g8pd_tests.log
[ $rc -ne 0 ] && exit $rc
for v in "DTC_GEMM8P=0" "DTC_GEMM8P=2" "DTC_GEMM8P=2 DTC_GEMM_SK=3"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --no-ref --only "fwd ,dgrad,wgrad lm_head" > gpurun_out/r3_g8pd_$tag.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r3_g8pd_$tag.log
done
