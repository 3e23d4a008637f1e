#!/bin/bash
# round 4, GPU call C: rewritten 32-row attention kernels (single register stage, buffer loads,
# diagonal-only masks): numerics tests, then an in-process A/B per dK/dV compile variant
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" > gpurun_out/r4c_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAIL" gpurun_out/r4c_tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
for v in default split1 all1; do
  if [ $v = default ]; then L=""; else L="variants/_dtc_$v.so"; fi
  echo "== $v" >> gpurun_out/r4c_ab.log
  DTC_KERNEL_LIB=$L $T 240 python benchmarks/attn_ab.py --rounds 5 >> gpurun_out/r4c_ab.log 2>&1 || exit $?
done
cat gpurun_out/r4c_ab.log
