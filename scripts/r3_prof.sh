#!/bin/bash
# kernel-trace profile of the default GPT-2 small step + summary
set -u
mkdir -p gpurun_out
bash scripts/prof_step.sh prof_cur || exit $?
python scripts/prof_summary.py gpurun_out/prof_cur/prof_kernel_trace.csv --out gpurun_out/prof_cur.md --title "GPT-2 small step (current default)" > /dev/null && cat gpurun_out/prof_cur.md
