#!/bin/bash
# round 4, GPU call J: fused grad-norm partials and the residual add moved into the LayerNorm pass
# (engine / kernel / wgrad tests), step A/B of both, then the whole-step PMC table and a kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_wgrad_group_gpu.py tests/test_kernels_gpu.py > gpurun_out/r4j_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAIL" gpurun_out/r4j_tests.log | tail -5; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_FUSED_NORM=1" "DTC_FUSED_NORM=0" "DTC_ADD_LN=0" || exit 1
bash scripts/pmc_step.sh || exit $?
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_j -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_j.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_j.log | cut -c1-200
