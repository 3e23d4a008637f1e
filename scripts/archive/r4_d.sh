#!/bin/bash
# round 4, GPU call D: gemm4w (layer GEMMs, 128x192 tiles, 2 blocks/CU) vs the shipped plans vs hipBLASLt
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/gemm_layer_ab.py --rounds 5 > gpurun_out/r4d_ab.log 2>&1; rc=$?
cat gpurun_out/r4d_ab.log | grep -v amdgpu.ids; exit $rc
