#!/bin/bash
# round 4, GPU call AD: the qkv forward on 256 x 192 tiles (DTC_BIG_CB3_FWD: 1.5 instead of 2 tile-times)
# -- numerics, in-step A/B, kernel trace
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_n8_gpu.py -k "cb3" > gpurun_out/r4ad_tests.log 2>&1 || { tail -40 gpurun_out/r4ad_tests.log; exit 1; }
tail -2 gpurun_out/r4ad_tests.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_BIG_CB3_FWD=1" > gpurun_out/r4ad_ab.log 2>&1 || { tail -20 gpurun_out/r4ad_ab.log; exit 1; }
cat gpurun_out/r4ad_ab.log
DTC_BIG_CB3_FWD=1 $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ad -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/r4ad_prof.log 2>&1 || { tail -30 gpurun_out/r4ad_prof.log; exit 1; }
echo prof done
