#!/bin/bash
# round 4, GPU call G: in-step A/B (whole GPT-2 small step, interleaved): gemm4w plan off / on, the
# comm-safe plans (what the DP backward runs under RCCL) at dp1, and the dp>1 wgrad grouping at dp1
set -u
export TMPDIR=/tmp
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_GEMM4W=0" "DTC_GEMM4W=1" "DTC_GEMM8N=0 DTC_WGRAD256=0" "|--set wgrad_group=2"
