#!/bin/bash
# round 4, GPU call P: CE backward rows per partial slab (DTC_CE_ROWS) in the step, CE tests, and a
# kernel trace of the current default step
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
DTC_CE_ROWS=128 $T 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lmhead or ce" > gpurun_out/r4p_tests.log 2>&1 || { tail -20 gpurun_out/r4p_tests.log; exit 1; }
tail -1 gpurun_out/r4p_tests.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "" "DTC_CE_ROWS=128" "DTC_CE_ROWS=256" || exit 1
cp gpurun_out/ab/summary.log gpurun_out/r4p_ab.log
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_p.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_p.log | cut -c1-160
