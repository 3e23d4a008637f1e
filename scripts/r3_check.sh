#!/bin/bash
# full GPU test suite + scaling-harness smoke (N=1 rows only on a 1-GPU box)
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3_gpu_all.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed" gpurun_out/r3_gpu_all.log | tail -n 3
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 900 bash scripts/scale_sweep.sh 10 3 > gpurun_out/r3_scale_sweep.log 2>&1; rc=$?
cat gpurun_out/r3_scale_sweep.log | tail -n 20
cp -r outputs gpurun_out/r3_outputs 2>/dev/null
exit $rc
