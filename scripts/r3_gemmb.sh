#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 > gpurun_out/r3_gemmb_g2s.log 2>&1 || exit $?
DTC_GEMM_W8=2 timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 > gpurun_out/r3_gemmb_g2s_w8.log 2>&1 || exit $?
DTC_BIG_MIN_TILES=128 timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 > gpurun_out/r3_gemmb_g2s_big.log 2>&1 || exit $?
paste gpurun_out/r3_gemmb_g2s.log gpurun_out/r3_gemmb_g2s_w8.log | cut -c1-200
