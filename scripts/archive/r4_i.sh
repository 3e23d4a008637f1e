#!/bin/bash
# round 4, GPU call I: P2P v3 (producer GEMM writes the bf16 partial into the IPC buffer half):
# multi-rank GPU tests (P2P unit + TP 2/4/8 on one GPU), then the P2P latency table at W = 2 and 4
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r4i_dist.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/r4i_dist.log | tail -20; [ $rc -ne 0 ] && exit $rc
$T 300 python benchmarks/p2p_bench.py --world 2 > gpurun_out/r4i_p2p_w2.log 2>&1 || exit $?
$T 300 python benchmarks/p2p_bench.py --world 4 > gpurun_out/r4i_p2p_w4.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r4i_p2p_w2.log gpurun_out/r4i_p2p_w4.log | grep -v Gloo
