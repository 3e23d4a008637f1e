#!/bin/bash
# Run one gpurun call; retry ONLY while no box/slot is free (exit code 3: nothing ran, nothing charged).
#   bash scripts/gpu_call.sh <tag> <timeout_s> '<command>'   -> gpurun_out/<tag>.txt
tag=$1; to=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "gpurun_out/$tag.txt" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "gpurun_out/$tag.txt"; then break; fi
  sleep 60
done
echo "rc=$rc" >> "gpurun_out/$tag.txt"
