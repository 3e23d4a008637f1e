#!/bin/bash
# round 4, GPU call AL: GPT-2 medium (d1024 L24 T1024) with the final round-4 code
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model gpt2-medium --steps 20 --warmup 3 > gpurun_out/r4al_medium.log 2>&1 || { tail -30 gpurun_out/r4al_medium.log; exit 1; }
grep '^{' gpurun_out/r4al_medium.log | cut -c1-260
