#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_X=0" "DTC_N8_GM=4" "DTC_N8_GM=16" "DTC_N8_GM=2"
