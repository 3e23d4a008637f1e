#!/bin/bash
set -u
timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 > gpurun_out/r3_gemmb_g2s_v2.log 2>&1 || exit $?
grep -E "qkv|out" gpurun_out/r3_gemmb_g2s_v2.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_BIG_TAIL=64" "DTC_BIG_TAIL=-1" "DTC_BIG_TAIL=64|--model ref" "DTC_BIG_TAIL=-1|--model ref"
