#!/bin/bash
# round 4, GPU call Y: grouped weight gradients with the last partial round split into K-pieces
# (DTC_WG_TAIL_SPLIT) -- group tests, fused-norm engine test with the split on, in-step A/B, kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wgrad_group_gpu.py > gpurun_out/r4y_tests.log 2>&1 || { tail -40 gpurun_out/r4y_tests.log; exit 1; }
tail -2 gpurun_out/r4y_tests.log
DTC_WG_TAIL_SPLIT=1 $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "fused_grad_norm or gpt2_small_step or graph_replay" > gpurun_out/r4y_tests2.log 2>&1 || { tail -40 gpurun_out/r4y_tests2.log; exit 1; }
tail -2 gpurun_out/r4y_tests2.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_WG_TAIL_SPLIT=1" > gpurun_out/r4y_ab.log 2>&1 || { tail -20 gpurun_out/r4y_ab.log; exit 1; }
cat gpurun_out/r4y_ab.log
DTC_WG_TAIL_SPLIT=1 $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_y -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4y_prof.log 2>&1 || { tail -30 gpurun_out/r4y_prof.log; exit 1; }
echo prof done
