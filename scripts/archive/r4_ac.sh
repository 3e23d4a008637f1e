#!/bin/bash
# round 4, GPU call AC: whole-step PMC counters of the final GPT-2 small step (three rocprofv3 --pmc
# passes within the per-pass budget, scripts/pmc_step.sh), each pass under its own time limit
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_TAG=final timeout -k 10 600 bash scripts/pmc_step.sh > gpurun_out/r4ac_pmc.log 2>&1 || { tail -30 gpurun_out/r4ac_pmc.log; exit 1; }
ls gpurun_out | grep pmc_final
