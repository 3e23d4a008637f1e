#!/bin/bash
# round 4, GPU call Q: rehearsal of the driver's N = 8 DP bench (8 processes sharing ONE GPU over gloo:
# exercises the dp > 1 step -- 2-layer weight-gradient groups, bucketed all-reduces, embedding-grad
# gather, comm-safe plans -- on the real kernels; its timing says nothing about 8 GPUs), and N = 2
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
DTC_DIST_BACKEND=gloo $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 2 > gpurun_out/r4q_dp2.log 2>&1 || { tail -30 gpurun_out/r4q_dp2.log; exit 1; }
grep '^{' gpurun_out/r4q_dp2.log | cut -c1-300
DTC_DIST_BACKEND=gloo $T 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 8 --steps 3 --warmup 2 > gpurun_out/r4q_dp8.log 2>&1 || { tail -30 gpurun_out/r4q_dp8.log; exit 1; }
grep '^{' gpurun_out/r4q_dp8.log | cut -c1-300
