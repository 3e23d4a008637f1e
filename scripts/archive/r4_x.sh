#!/bin/bash
# round 4, GPU call X: lm_head dgrad on 256 x 192 split-K tiles (DTC_BIG_CB3: 256 blocks instead of 192)
# -- numerics test, in-step interleaved A/B; embedding stage-1 block order (piece sums first) rides along
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_n8_gpu.py tests/test_kernels_gpu.py -k "cb3 or embed" > gpurun_out/r4x_tests.log 2>&1 || { tail -40 gpurun_out/r4x_tests.log; exit 1; }
tail -2 gpurun_out/r4x_tests.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_BIG_CB3=1" > gpurun_out/r4x_ab.log 2>&1 || { tail -20 gpurun_out/r4x_ab.log; exit 1; }
cat gpurun_out/r4x_ab.log
DTC_BIG_CB3=1 $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4x_prof.log 2>&1 || { tail -30 gpurun_out/r4x_prof.log; exit 1; }
echo prof done
