#!/bin/bash
# lm_head dgrad split-K A/B (DTC_CE_SPLIT) + correctness of the split variants
set -u
mkdir -p gpurun_out
DTC_CE_SPLIT=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "ce or lmhead or xent" > gpurun_out/ce_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/ce_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_CE_SPLIT=0" "DTC_CE_SPLIT=5" "DTC_CE_SPLIT=8" "DTC_CE_SPLIT=4"
