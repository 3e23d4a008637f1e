#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python scripts/rehearse_medium.py --steps 3 --batch 4 > gpurun_out/r3_rehearse_medium.log 2>&1; rc=$?
tail -n 25 gpurun_out/r3_rehearse_medium.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 bash scripts/multirank_smoke.sh > gpurun_out/r3_multirank.log 2>&1; rc=$?
cat gpurun_out/r3_multirank.log
exit $rc
