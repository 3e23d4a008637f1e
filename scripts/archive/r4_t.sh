#!/bin/bash
# round 4, GPU call T: debug-build (device asserts live) GPT-2-small-shaped steps vs release,
# kernel tests after the assert additions, 1-GPU bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 700 --timeout-method thread tests/test_debug_build_gpu.py tests/test_kernels_gpu.py tests/test_dist_gpu.py > gpurun_out/r4t_tests.log 2>&1 || { tail -40 gpurun_out/r4t_tests.log; exit 1; }
tail -3 gpurun_out/r4t_tests.log
$T 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r4t_bench.log 2>&1 || { tail -30 gpurun_out/r4t_bench.log; exit 1; }
grep '^{' gpurun_out/r4t_bench.log | cut -c1-300
