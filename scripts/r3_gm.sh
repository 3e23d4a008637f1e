#!/bin/bash
set -u
mkdir -p gpurun_out
for g in 0 8; do
  DTC_WIDE_GM=$g timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --no-ref --only fc1,fc2,lm_head > gpurun_out/gm_bench$g.log 2>&1 || exit $?
done
paste gpurun_out/gm_bench0.log gpurun_out/gm_bench8.log | cut -c1-150
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_WIDE_GM=0" "DTC_WIDE_GM=8" "DTC_WIDE_GM=4" "DTC_WIDE_GM=16"
