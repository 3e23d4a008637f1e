#!/bin/bash
# round 4, GPU call E: gemm4w / gemm4p A/B with and without VGPR-form MFMAs (-mllvm -amdgpu-mfma-vgpr-form),
# then the step with each library (does the flag cost the other kernels anything?)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4w_gpu.py > gpurun_out/r4e_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4e_tests.log; [ $rc -ne 0 ] && exit $rc
DTC_KERNEL_LIB=variants/_dtc_vgprform.so $T 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4w_gpu.py > gpurun_out/r4e_tests_v.log 2>&1; rc=$?
tail -3 gpurun_out/r4e_tests_v.log; [ $rc -ne 0 ] && exit $rc
echo "== in-tree" > gpurun_out/r4e_ab.log
$T 300 python benchmarks/gemm_layer_ab.py --rounds 5 2>&1 | grep -v check >> gpurun_out/r4e_ab.log || exit 1
echo "== vgpr-form" >> gpurun_out/r4e_ab.log
DTC_KERNEL_LIB=variants/_dtc_vgprform.so $T 300 python benchmarks/gemm_layer_ab.py --rounds 5 2>&1 | grep -v check >> gpurun_out/r4e_ab.log || exit 1
cat gpurun_out/r4e_ab.log
for i in 1 2; do
  $T 200 python bench.py --steps 20 --warmup 5 2>&1 | grep '^{' | tail -1 | cut -c1-200
  DTC_KERNEL_LIB=variants/_dtc_vgprform.so $T 200 python bench.py --steps 20 --warmup 5 2>&1 | grep '^{' | tail -1 | cut -c1-200
done
