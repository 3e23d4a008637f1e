#!/bin/bash
set -u
mkdir -p gpurun_out
ROUNDS=3 STEPS=30 bash scripts/ab_bench.sh "DTC_WIDE_GM=4" "DTC_WIDE_GM=2" "DTC_WIDE_GM=3" || exit $?
PMC_TAG=cur bash scripts/pmc_step.sh || exit $?
python scripts/pmc_summary.py gpurun_out --tag cur --out gpurun_out/pmc_cur.md --title "GPT-2 small step, round-3 final kernels: hardware counters (rocprofv3 --pmc, 3 passes)" > /dev/null && head -12 gpurun_out/pmc_cur.md
