#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_X=0" "DTC_VOCAB_SPLIT=5" "DTC_VOCAB_SPLIT=8" "DTC_VOCAB_SPLIT=3"
