#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=2 STEPS=50 bash scripts/ab_bench.sh "DTC_X=0|--model ref" "DTC_LN_FUSE=0|--model ref" "DTC_CE_FUSED=0|--model ref" "DTC_SIDE_STREAM=1|--model ref" "DTC_LN_FUSE=3|--model ref"
