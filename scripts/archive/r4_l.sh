#!/bin/bash
# round 4, GPU call L: in-step A/B of the multi-round layer-GEMM plans (gemm8n on 3-4 round grids:
# qkv / fc1 forwards, fc2 dgrad) and the qkv forward off the 256^2 tail plan
set -u
export TMPDIR=/tmp
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "" "DTC_GEMM8N=7" "DTC_BIG_TAIL=0" || exit 1
cp gpurun_out/ab/summary.log gpurun_out/r4l_ab.log
