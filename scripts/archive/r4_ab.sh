#!/bin/bash
# round 4, GPU call AB: out_proj forward / NT dgrad (K = 768, 256 tiles of 128 x 192) on the persistent gemm8n
# kernel (DTC_N8_MINK=768) -- cold per-shape table, numerics, in-step A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python benchmarks/gemm_layer_ab.py --cold --rounds 5 --reps 20 --only "fwd out,ntdgrad out" --variants n8k768 > gpurun_out/r4ab_gemm.log 2>&1 || { tail -20 gpurun_out/r4ab_gemm.log; exit 1; }
grep -v "amdgpu.ids" gpurun_out/r4ab_gemm.log
rm -f gpurun_out/ab/summary.log
ROUNDS=3 STEPS=40 $T 900 bash scripts/ab_bench.sh "" "DTC_N8_MINK=768" > gpurun_out/r4ab_ab.log 2>&1 || { tail -20 gpurun_out/r4ab_ab.log; exit 1; }
cat gpurun_out/r4ab_ab.log
