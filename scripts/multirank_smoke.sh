#!/bin/bash
# The driver's multi-GPU bench command, rehearsed with 2 ranks on ONE GPU (gloo: RCCL refuses two
# ranks per device) for dp / tp / pp: validates the multi-rank bench path end to end (not its speed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export DTC_DIST_BACKEND=gloo
port=29610
for par in dp tp pp; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 5 --warmup 2 --parallel $par > gpurun_out/mr_$par.log 2>&1 || exit $?
  grep '"metric"' gpurun_out/mr_$par.log | cut -c1-200
done
# hybrid DP x TP (BASELINE config 5's mesh shape at 4 ranks: dp2 x tp2)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port $((port + 1)) bench.py --gpus 4 --steps 5 --warmup 2 --parallel dp --tp 2 > gpurun_out/mr_hyb.log 2>&1 || exit $?
grep '"metric"' gpurun_out/mr_hyb.log | cut -c1-200
