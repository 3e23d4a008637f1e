#!/bin/bash
# round 4, GPU call AG: one-pass CE row combine -- kernel / engine / dist tests, bench, kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_dist_gpu.py > gpurun_out/r4ag_tests.log 2>&1 || { tail -40 gpurun_out/r4ag_tests.log; exit 1; }
tail -2 gpurun_out/r4ag_tests.log
$T 300 python bench.py --steps 50 --warmup 5 > gpurun_out/r4ag_bench.log 2>&1 || { tail -30 gpurun_out/r4ag_bench.log; exit 1; }
grep '^{' gpurun_out/r4ag_bench.log | cut -c1-300
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ag -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4ag_prof.log 2>&1 || { tail -30 gpurun_out/r4ag_prof.log; exit 1; }
echo prof done
