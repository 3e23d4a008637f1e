#!/bin/bash
# round 4, GPU call U: bf16 branch outputs (DTC_FWD_BF16 / DTC_DGRAD_BF16) -- kernel + engine tests,
# then an interleaved in-step A/B of the two knobs
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "add_layernorm" tests/test_engine_gpu.py::test_bf16_branch_outputs_match tests/test_engine_gpu.py::test_gpt2_small_step_vs_oracle > gpurun_out/r4u_tests.log 2>&1 || { tail -40 gpurun_out/r4u_tests.log; exit 1; }
tail -2 gpurun_out/r4u_tests.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_FWD_BF16=1" "DTC_DGRAD_BF16=1" "DTC_FWD_BF16=1 DTC_DGRAD_BF16=1" > gpurun_out/r4u_ab.log 2>&1 || { tail -20 gpurun_out/r4u_ab.log; exit 1; }
cat gpurun_out/r4u_ab.log
