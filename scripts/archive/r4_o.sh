#!/bin/bash
# round 4, GPU call O: LayerNorm-backward partial rows (DTC_LN_BWD_ITER) and the lm_head dgrad on the
# untransposed weight (DTC_DGRAD_NT_HEAD=0: no transpose of the 38.6 M-element weight per step)
set -u
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k layernorm > gpurun_out/r4o_tests.log 2>&1 || { tail -20 gpurun_out/r4o_tests.log; exit 1; }
DTC_LN_BWD_ITER=4 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k layernorm >> gpurun_out/r4o_tests.log 2>&1 || { tail -20 gpurun_out/r4o_tests.log; exit 1; }
grep passed gpurun_out/r4o_tests.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "" "DTC_LN_BWD_ITER=2" "DTC_LN_BWD_ITER=4" "DTC_DGRAD_NT_HEAD=0" || exit 1
cp gpurun_out/ab/summary.log gpurun_out/r4o_ab.log
