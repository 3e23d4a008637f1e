#!/bin/bash
# gemm8n on one-round shapes: tests, whole-step A/B, kernel-trace profile of the default
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_n8_gpu.py > gpurun_out/n8_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/n8_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM8N=0" "DTC_GEMM8N=3" || exit $?
bash scripts/prof_step.sh prof_n8 || exit $?
python scripts/prof_summary.py gpurun_out/prof_n8/prof_kernel_trace.csv --out gpurun_out/prof_n8.md --title "GPT-2 small step, gemm8n" > /dev/null && head -40 gpurun_out/prof_n8.md
