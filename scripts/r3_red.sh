#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "reducer or wgrad or colsum" > gpurun_out/red_tests.log 2>&1; rc=$?
tail -n 2 gpurun_out/red_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/prof_step.sh prof_red || exit $?
python scripts/prof_summary.py gpurun_out/prof_red/prof_kernel_trace.csv --out gpurun_out/prof_red.md --title "GPT-2 small step, unrolled slab reduce" > /dev/null && grep -E "GPU-busy|reduce_tasks" gpurun_out/prof_red.md
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_X=0"
