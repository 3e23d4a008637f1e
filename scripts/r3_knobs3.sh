#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_X=0" "DTC_DGRAD_NT_FC2=1" "DTC_BK128=32" "DTC_GEMM_DMA=5" "DTC_GEMM_DMA=5 DTC_DMA_STAGES128=3"
