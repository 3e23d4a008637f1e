#!/bin/bash
# round 4, GPU call V: bf16-branch engine test; cold per-shape GEMM table with the diagnostic rows
# (fc1 forward with one plain output, bf16 dgrad / forward outputs) vs hipBLASLt
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py::test_bf16_branch_outputs_match > gpurun_out/r4v_tests.log 2>&1 || { tail -40 gpurun_out/r4v_tests.log; exit 1; }
tail -2 gpurun_out/r4v_tests.log
$T 600 python benchmarks/gemm_layer_ab.py --cold --rounds 5 --reps 20 > gpurun_out/r4v_gemm_cold.log 2>&1 || { tail -20 gpurun_out/r4v_gemm_cold.log; exit 1; }
grep -v "^check" gpurun_out/r4v_gemm_cold.log
