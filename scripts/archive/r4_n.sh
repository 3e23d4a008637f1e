#!/bin/bash
# round 4, GPU call N: full GPU test suite, smoke and bench on the current tree (verification after the
# fused norm, residual-in-LN, merged attention backward and P2P staging changes)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4n_gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4n_gpu_tests.log | tail -2; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r4n_gpu_tests.log | head; exit $rc; }
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r4n_smoke.log
$T 300 python bench.py > gpurun_out/r4n_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r4n_bench.log
