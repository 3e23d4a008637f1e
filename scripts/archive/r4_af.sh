#!/bin/bash
# round 4, GPU call AF: the layers' LayerNorm / bias partial reductions batched into the grouped
# weight-gradient flush (DTC_RED_BATCH_LAYERS; reduce batches of up to 48 tasks) -- engine tests with it,
# in-step A/B, kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
DTC_RED_BATCH_LAYERS=1 $T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_wgrad_group_gpu.py > gpurun_out/r4af_tests.log 2>&1 || { tail -40 gpurun_out/r4af_tests.log; exit 1; }
tail -2 gpurun_out/r4af_tests.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_RED_BATCH_LAYERS=1" > gpurun_out/r4af_ab.log 2>&1 || { tail -20 gpurun_out/r4af_ab.log; exit 1; }
cat gpurun_out/r4af_ab.log
DTC_RED_BATCH_LAYERS=1 $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_af -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4af_prof.log 2>&1 || { tail -30 gpurun_out/r4af_prof.log; exit 1; }
echo prof done
