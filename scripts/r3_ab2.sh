#!/bin/bash
set -u
ROUNDS=2 STEPS=30 bash scripts/ab_bench.sh "DTC_X=0" "|--set defer_optimizer=true" "DTC_SIDE_STREAM=1" "DTC_CE_FUSED=0" "DTC_DGRAD_NT=0" "DTC_DGRAD_NT_FC2=1" "DTC_GEMM_PAIR=0" > gpurun_out/r3_ab2.log 2>&1
cat gpurun_out/r3_ab2.log
