#!/bin/bash
# round 4, GPU call H: layer-GEMM A/B with cold caches (512 MB write before every call), in-tree and
# VGPR-form MFMA builds: does the cold harness reproduce the in-step ranking?
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
echo "== in-tree cold" > gpurun_out/r4h_ab.log
$T 400 python benchmarks/gemm_layer_ab.py --cold --rounds 3 2>&1 | grep -v "check\|amdgpu" >> gpurun_out/r4h_ab.log || exit 1
echo "== vgpr-form cold" >> gpurun_out/r4h_ab.log
DTC_KERNEL_LIB=variants/_dtc_vgprform.so $T 400 python benchmarks/gemm_layer_ab.py --cold --rounds 3 2>&1 | grep -v "check\|amdgpu" >> gpurun_out/r4h_ab.log || exit 1
cat gpurun_out/r4h_ab.log
