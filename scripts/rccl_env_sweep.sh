#!/bin/bash
# RCCL channel / algorithm / protocol sweep for the DP gradient all-reduce on one 8 x MI355X node
# (a ring uses one outgoing xGMI link per GPU, so the channel count decides how many of
# the 7 links a collective drives).  Runs bench.py --parallel dp at N GPUs under each setting and
# prints ms/step; the fastest setting goes into the launch environment.
#
#   bash scripts/rccl_env_sweep.sh [N=8] [STEPS=20]       (needs N visible GPUs; skipped otherwise)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-8}
STEPS=${2:-20}
NGPU=$(python -c "import torch; print(torch.cuda.device_count())")
if [ "$N" -gt "$NGPU" ]; then echo "skip: $N GPUs requested, $NGPU visible"; exit 0; fi
mkdir -p outputs/rccl_sweep
PORT=29700
for setting in "" "NCCL_MIN_NCHANNELS=16" "NCCL_MIN_NCHANNELS=32" "NCCL_MIN_NCHANNELS=64" \
               "NCCL_ALGO=Ring" "NCCL_ALGO=Tree" "NCCL_PROTO=Simple" "NCCL_PROTO=LL128" \
               "NCCL_MIN_NCHANNELS=32 NCCL_PROTO=Simple"; do
  PORT=$((PORT + 1))
  tag=$(echo "${setting:-default}" | tr ' =' '_-')
  # shellcheck disable=SC2086
  env $setting timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus $N --steps $STEPS --warmup 5 \
      > outputs/rccl_sweep/$tag.log 2>&1
  rc=$?
  ms=$(grep -o '"ms_per_step": [0-9.]*' outputs/rccl_sweep/$tag.log | awk '{print $2}')
  echo "${setting:-default}: rc=$rc ms_per_step=${ms:-n/a}" | tee -a outputs/rccl_sweep/summary.log
  case $rc in 124|137|134|139) echo "stopping: hang or crash"; exit $rc ;; esac
done
