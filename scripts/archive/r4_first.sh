#!/bin/bash
# round-4 first GPU call: re-baseline GPT-2 small, and the comm-safe GEMM plans forced on at dp1
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r4_base.log 2>&1 || exit $?
tail -n 1 gpurun_out/r4_base.log
DTC_GEMM8N=0 DTC_WGRAD256=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r4_commsafe.log 2>&1 || exit $?
tail -n 1 gpurun_out/r4_commsafe.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r4_base2.log 2>&1 || exit $?
tail -n 1 gpurun_out/r4_base2.log
