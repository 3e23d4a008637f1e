#!/bin/bash
# whole-step knob A/B on the gemm8n build, then the full GPU suite
set -u
mkdir -p gpurun_out
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_X=0" "DTC_SIDE_STREAM=1" "DTC_SIDE_STREAM=1 DTC_GEMM8N=0 DTC_WGRAD256=0" "DTC_CE_FUSED=0" || exit $?
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_all.log 2>&1; rc=$?
tail -n 5 gpurun_out/gpu_all.log
exit $rc
