#!/bin/bash
# round 4, GPU call W: embedding backward in two launches (table zeroing + piece sums + dwpe in one grid)
# -- the whole GPU suite, smoke, 1-GPU bench, kernel trace; cold GEMM table of the multi-round gemm8n plans
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4w_tests.log 2>&1 || { tail -40 gpurun_out/r4w_tests.log; exit 1; }
tail -2 gpurun_out/r4w_tests.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4w_smoke.log 2>&1 || { tail -20 gpurun_out/r4w_smoke.log; exit 1; }
tail -1 gpurun_out/r4w_smoke.log
$T 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r4w_bench.log 2>&1 || { tail -30 gpurun_out/r4w_bench.log; exit 1; }
grep '^{' gpurun_out/r4w_bench.log | cut -c1-300
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4w_prof.log 2>&1 || { tail -30 gpurun_out/r4w_prof.log; exit 1; }
echo prof done
$T 600 python benchmarks/gemm_layer_ab.py --cold --rounds 5 --reps 20 --only "fwd qkv,fwd fc1,ntdgrad fc2" --variants n8,n8w3,n8w4 > gpurun_out/r4w_gemm_n8.log 2>&1 || { tail -20 gpurun_out/r4w_gemm_n8.log; exit 1; }
grep -v "^check" gpurun_out/r4w_gemm_n8.log
