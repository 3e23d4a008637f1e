#!/bin/bash
# Kernel-trace profile of bench.py (one rocprofv3 run): bash scripts/prof_step.sh <outname> [bench args...]
# Writes gpurun_out/<outname>/prof_kernel_trace.csv (+ stats).  Extra env (A/B knobs) is inherited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o prof --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --ref32 off "$@" > "gpurun_out/$name.log" 2>&1
