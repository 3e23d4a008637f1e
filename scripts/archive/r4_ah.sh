#!/bin/bash
# round 4, GPU call AH: attention delta from the out_proj dgrad's epilogue (DTC_DELTA_EPI) -- kernel and
# engine tests, in-step A/B, kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "delta or attention or lmhead" tests/test_engine_gpu.py::test_delta_epilogue_matches > gpurun_out/r4ah_tests.log 2>&1 || { tail -40 gpurun_out/r4ah_tests.log; exit 1; }
tail -2 gpurun_out/r4ah_tests.log
DTC_DELTA_EPI=1 $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "gpt2_small_step or graph_replay or fused_grad_norm" > gpurun_out/r4ah_tests2.log 2>&1 || { tail -40 gpurun_out/r4ah_tests2.log; exit 1; }
tail -2 gpurun_out/r4ah_tests2.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_DELTA_EPI=1" > gpurun_out/r4ah_ab.log 2>&1 || { tail -20 gpurun_out/r4ah_ab.log; exit 1; }
cat gpurun_out/r4ah_ab.log
DTC_DELTA_EPI=1 $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ah -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4ah_prof.log 2>&1 || { tail -30 gpurun_out/r4ah_prof.log; exit 1; }
echo prof done
