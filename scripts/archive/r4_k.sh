#!/bin/bash
# round 4, GPU call K: merged attention backward (tests + A/B in process and in the step), the multi-rank
# GPU tests with the fused grad norm on (TP at dp 1), cold layer-GEMM table as the step runs them
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "attn or attention or fused_grad_norm" > gpurun_out/r4k_attn_tests.log 2>&1 || { tail -30 gpurun_out/r4k_attn_tests.log; exit 1; }
tail -1 gpurun_out/r4k_attn_tests.log
$T 240 python benchmarks/attn_ab.py --rounds 5 2>&1 | grep -v amdgpu | tee gpurun_out/r4k_attn_ab.log || exit 1
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r4k_dist.log 2>&1 || { tail -30 gpurun_out/r4k_dist.log; exit 1; }
tail -1 gpurun_out/r4k_dist.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_ATTN_BWD_MERGED=0" "DTC_ATTN_BWD_MERGED=1" || exit 1
cp gpurun_out/ab/summary.log gpurun_out/r4k_ab_merged.log
$T 400 python benchmarks/gemm_layer_ab.py --cold --rounds 3 2>&1 | grep -v "check\|amdgpu" > gpurun_out/r4k_gemm_cold.log || exit 1
cat gpurun_out/r4k_gemm_cold.log
