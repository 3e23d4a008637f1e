#!/bin/bash
# TP=8 rehearsal: 8 ranks of bench.py --parallel tp on ONE GPU (gloo bootstrap, the in-graph P2P kernels for
# every TP collective), each layout under rocprofv3 --kernel-trace: per-rank kernel sums by class
# (scripts/tp_rehearsal_report.py).  Timing is not the 8-GPU number (8 processes share one device, the
# P2P barrier kernels spin while peers run); the per-rank compute-kernel sums and launch counts are.
#   bash scripts/tp8_rehearsal.sh  -> gpurun_out/tp8_<name>/ + gpurun_out/tp8_<name>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export DTC_DIST_BACKEND=gloo
port=29710
run() {
  name=$1; shift
  port=$((port + 1))
  # each rank runs under its own profiler (the launcher never touches the GPU; rocprofv3 starts the rank)
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $port --no-python rocprofv3 --kernel-trace -d "gpurun_out/tp8_$name" --output-format csv -- \
    python bench.py --gpus 8 --parallel tp --steps 4 --warmup 2 --set tp_comm=p2p "$@" > "gpurun_out/tp8_$name.log" 2>&1
}
run fp32 && run bf16 --set tp_comm_dtype=bf16 && run sp_bf16 --set tp_comm_dtype=bf16 --set tp_sequence_parallel=true
