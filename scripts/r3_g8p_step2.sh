#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM8P=2" "DTC_GEMM8P=0"
