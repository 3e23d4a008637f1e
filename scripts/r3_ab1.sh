#!/bin/bash
set -u
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_X=0" "DTC_GEMM_W8=2" "DTC_BIG_MIN_TILES=256" "DTC_BIG_MIN_TILES=128" "DTC_GEMM_W8=3" "DTC_WGRAD_BLOCKS=512" "DTC_GEMM_DMA=5" > gpurun_out/r3_ab1.log 2>&1
cat gpurun_out/r3_ab1.log
