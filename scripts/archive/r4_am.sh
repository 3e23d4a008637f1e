#!/bin/bash
# round 4, GPU call AM: re-check two reduction-granularity knobs under the final defaults (in-step A/B)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 timeout -k 10 900 bash scripts/ab_bench.sh "" "DTC_LN_BWD_ITER=4" "DTC_CE_ROWS=64" > gpurun_out/r4am_ab.log 2>&1 || { tail -20 gpurun_out/r4am_ab.log; exit 1; }
cat gpurun_out/r4am_ab.log
