#!/bin/bash
# round 4, GPU call F: the whole GPU test suite, smoke, bench, a kernel trace of the step, then the
# cross-strategy long curves (dp1 / tp2 P2P / pp2 1F1B on one GPU)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4f_gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4f_gpu_tests.log | tail -2; [ $rc -ne 0 ] && exit $rc
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r4f_smoke.log
$T 300 python bench.py > gpurun_out/r4f_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r4f_bench.log | cut -c1-220
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_f.log 2>&1 || exit $?
STEPS=2000 bash scripts/cross_strategy_runs.sh
