#!/bin/bash
# round 4, GPU call A: grouped weight gradients (kernel + engine tests, step A/B), uneven-head TP and
# dp2 x tp2 at the default HW queue count, GPT-2 small TP=8 rehearsal (8 processes on one GPU)
set -u
mkdir -p gpurun_out
T="timeout -k 10"
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_group_gpu.py tests/test_gemm_n8_gpu.py tests/test_kernels_gpu.py -k "wgrad or n8 or split256 or attention" > gpurun_out/r4_wg_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r4_wg_tests.log; [ $rc -ne 0 ] && exit $rc
$T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py > gpurun_out/r4_wg_engine.log 2>&1; rc=$?
tail -n 3 gpurun_out/r4_wg_engine.log; [ $rc -ne 0 ] && exit $rc
$T 300 python benchmarks/attn_ab.py --rounds 5 > gpurun_out/r4_attn_ab.log 2>&1; tail -n 6 gpurun_out/r4_attn_ab.log
for arm in 0 -1 0; do
  $T 300 python bench.py --steps 30 --warmup 5 --set wgrad_group=$arm > gpurun_out/r4_wg_bench_$arm.log 2>&1 || exit $?
  echo "wgrad_group=$arm"; tail -n 1 gpurun_out/r4_wg_bench_$arm.log
done
DTC_GEMM8N=0 DTC_WGRAD256=0 $T 300 python bench.py --steps 30 --warmup 5 --set wgrad_group=-1 > gpurun_out/r4_commsafe.log 2>&1 || exit $?
echo "comm-safe plans at dp1 (old path)"; tail -n 1 gpurun_out/r4_commsafe.log
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py -k "uneven" > gpurun_out/r4_dist_uneven.log 2>&1; rc=$?
tail -n 4 gpurun_out/r4_dist_uneven.log; [ $rc -ne 0 ] && exit $rc
DTC_DIST_BACKEND=gloo $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --parallel tp --steps 3 --warmup 2 --set tp_comm=p2p > gpurun_out/r4_tp8_rehearsal.log 2>&1; rc=$?
grep '^{' gpurun_out/r4_tp8_rehearsal.log | tail -n 1; tail -n 2 gpurun_out/r4_tp8_rehearsal.log; exit $rc
