#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --model gpt2-medium --steps 20 --warmup 3 > gpurun_out/med.log 2>&1 || exit $?
tail -n 1 gpurun_out/med.log | cut -c1-400
timeout -k 10 400 env DTC_GEMM8N=0 DTC_WGRAD256=0 DTC_WIDE_GM=0 python bench.py --model gpt2-medium --steps 20 --warmup 3 > gpurun_out/med0.log 2>&1 || exit $?
tail -n 1 gpurun_out/med0.log | cut -c1-400
timeout -k 10 300 python bench.py --parallel pp --steps 20 --warmup 3 > gpurun_out/pp1.log 2>&1 || exit $?
tail -n 1 gpurun_out/pp1.log | cut -c1-300
