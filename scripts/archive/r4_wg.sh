#!/bin/bash
# grouped weight gradients: kernel tests, engine tests, then the GPT-2 small step A/B
set -u
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_group_gpu.py tests/test_gemm_n8_gpu.py > gpurun_out/r4_wg_tests.log 2>&1; rc=$?
tail -n 5 gpurun_out/r4_wg_tests.log; [ $rc -ne 0 ] && exit $rc
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py > gpurun_out/r4_wg_engine.log 2>&1; rc=$?
tail -n 5 gpurun_out/r4_wg_engine.log; [ $rc -ne 0 ] && exit $rc
for arm in 0 -1 0; do
  $T 300 python bench.py --steps 30 --warmup 5 --set wgrad_group=$arm > gpurun_out/r4_wg_bench_$arm.log 2>&1 || exit $?
  echo "wgrad_group=$arm"; tail -n 1 gpurun_out/r4_wg_bench_$arm.log
done
DTC_GEMM8N=0 DTC_WGRAD256=0 $T 300 python bench.py --steps 30 --warmup 5 --set wgrad_group=-1 > gpurun_out/r4_commsafe.log 2>&1 || exit $?
echo "comm-safe plans at dp1 (old path)"; tail -n 1 gpurun_out/r4_commsafe.log
