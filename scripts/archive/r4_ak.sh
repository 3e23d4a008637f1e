#!/bin/bash
# round 4, GPU call AK: the reference's own 89.6M model with the final round-4 code, bf16 and exact fp32
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python bench.py --model ref --steps 50 --warmup 5 > gpurun_out/r4ak_ref.log 2>&1 || { tail -30 gpurun_out/r4ak_ref.log; exit 1; }
grep '^{' gpurun_out/r4ak_ref.log | cut -c1-260
$T 300 python bench.py --model ref --set dtype=fp32 --steps 20 --warmup 3 > gpurun_out/r4ak_ref32.log 2>&1 || { tail -30 gpurun_out/r4ak_ref32.log; exit 1; }
grep '^{' gpurun_out/r4ak_ref32.log | cut -c1-260
