#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_f32_gpu.py -m gpu > gpurun_out/r3_f32_kernels.log 2>&1; rc=$?
echo "kernels rc=$rc"; tail -n 3 gpurun_out/r3_f32_kernels.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --model ref --steps 30 --warmup 3 --set dtype=fp32 > gpurun_out/r3_f32_bench_ref.log 2>&1 || exit $?
tail -n 1 gpurun_out/r3_f32_bench_ref.log
BENCH_ARGS="--model ref --set dtype=fp32" PMC_TAG=fp32 bash scripts/pmc_step.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_f32_prof -o prof --output-format csv -- python bench.py --model ref --steps 6 --warmup 3 --set dtype=fp32 > gpurun_out/r3_f32_prof.log 2>&1 || exit $?
echo ALLDONE
