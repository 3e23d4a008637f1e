#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=2 STEPS=50 bash scripts/ab_bench.sh "DTC_X=0|--model ref" "DTC_X=0"
