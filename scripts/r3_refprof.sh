#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref -o prof --output-format csv -- python bench.py --model ref --steps 10 --warmup 3 > gpurun_out/prof_ref.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_ref/prof_kernel_trace.csv --out gpurun_out/prof_ref.md --title "Reference model step (d512 L12 T512 B8), round-3 final" > /dev/null && head -40 gpurun_out/prof_ref.md
timeout -k 10 300 python benchmarks/gemm_bench.py --model ref --reps 30 > gpurun_out/gemm_ref.log 2>&1 || exit $?
cat gpurun_out/gemm_ref.log
