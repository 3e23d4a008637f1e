#!/bin/bash
# record pass without collectives + cross-rank sequence verification: multi-rank GPU tests, engine, bench
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_engine_gpu.py -m gpu > gpurun_out/r3_record_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 gpurun_out/r3_record_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3_record_bench.log 2>&1; rc=$?
tail -n 1 gpurun_out/r3_record_bench.log; exit $rc
