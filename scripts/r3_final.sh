#!/bin/bash
# round-3 final check: full GPU suite, smoke, bench (driver contract), step profile
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/final_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
tail -n 2 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/final_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/final_bench.log
timeout -k 10 300 python bench.py --model ref --steps 50 --warmup 5 > gpurun_out/final_bench_ref.log 2>&1 || exit $?
tail -n 1 gpurun_out/final_bench_ref.log
bash scripts/prof_step.sh prof_final || exit $?
python scripts/prof_summary.py gpurun_out/prof_final/prof_kernel_trace.csv --out gpurun_out/prof_final.md --title "GPT-2 small step, round-3 final" > /dev/null && head -30 gpurun_out/prof_final.md
