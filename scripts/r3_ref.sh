#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=2 STEPS=50 bash scripts/ab_bench.sh "DTC_X=0|--model ref" "DTC_WGRAD256=0|--model ref" "DTC_WIDE_GM=0|--model ref" "DTC_WGRAD256=0 DTC_WIDE_GM=0|--model ref" "DTC_WGRAD_CS256=0|--model ref"
