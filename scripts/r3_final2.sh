#!/bin/bash
# round-3 closing check: full GPU suite, smoke, bench (driver contract) for GPT-2 small and the reference model
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final2_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/final2_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2_smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/final2_smoke.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/final2_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/final2_bench.log | cut -c1-260
timeout -k 10 300 python bench.py --model ref --steps 50 --warmup 5 > gpurun_out/final2_bench_ref.log 2>&1 || exit $?
tail -n 1 gpurun_out/final2_bench_ref.log | cut -c1-260
