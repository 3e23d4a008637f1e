#!/bin/bash
# round 4, GPU call AA: whole-tile 256^2 forwards with a nearly empty last round split into K-pieces
# (DTC_BIG_TAIL_SPLIT: the qkv forward's 32 tail tiles x 4) -- numerics test, in-step A/B, trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_n8_gpu.py -k "tail or cb3" > gpurun_out/r4aa_tests.log 2>&1 || { tail -40 gpurun_out/r4aa_tests.log; exit 1; }
tail -2 gpurun_out/r4aa_tests.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_BIG_TAIL_SPLIT=1" > gpurun_out/r4aa_ab.log 2>&1 || { tail -20 gpurun_out/r4aa_ab.log; exit 1; }
cat gpurun_out/r4aa_ab.log
DTC_BIG_TAIL_SPLIT=1 $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aa -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4aa_prof.log 2>&1 || { tail -30 gpurun_out/r4aa_prof.log; exit 1; }
echo prof done
