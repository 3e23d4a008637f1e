#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm or ln" > gpurun_out/lnf_tests.log 2>&1; rc=$?
tail -n 2 gpurun_out/lnf_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_LN_FWD_RPW=1" "DTC_LN_FWD_RPW=2"
