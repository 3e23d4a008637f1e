#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k chunked > gpurun_out/chunk_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/chunk_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_CE_CHUNK=0" "DTC_CE_CHUNK=8192" "DTC_CE_CHUNK=16384"
