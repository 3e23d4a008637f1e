#!/bin/bash
# Scaling sweep on ONE node: bench.py at 1/2/4/8 GPUs for DP, TP and PP (GPT-2 small, the model
# BASELINE.json names), plus BASELINE.json config 5 (GPT-2 medium, dp4 x tp2 on 8 GPUs).
#
#   bash scripts/scale_sweep.sh [STEPS] [WARMUP]        (N > visible GPUs are skipped)
#   -> outputs/scaling_raw.jsonl (one bench JSON line per run), outputs/scaling.json (plot.py),
#      outputs/scaling.md (tokens/s, ms/step and efficiency vs N=1, per strategy)
#
# Every run is one torchrun with one rank per GPU over RCCL (127.0.0.1 rendezvous), under its own
# time limit; a run that fails or times out is recorded as failed and the sweep goes on to the
# next strategy only if the failure was not a hang/crash (exit 124/137/134/139 stop the sweep).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=${1:-20}
WARMUP=${2:-5}
OUT=outputs
mkdir -p $OUT
RAW=$OUT/scaling_raw.jsonl
: > $RAW
NGPU=$(python -c "import torch; print(torch.cuda.device_count())")
PORT=29611
run() {  # tag nproc args...
  local tag=$1 n=$2; shift 2
  if [ "$n" -gt "$NGPU" ]; then echo "skip $tag (N=$n > $NGPU GPUs)"; return 0; fi
  PORT=$((PORT + 1))
  local log=$OUT/scale_${tag}.log
  if [ "$n" -eq 1 ]; then
    timeout -k 10 600 python bench.py --gpus 1 --steps $STEPS --warmup $WARMUP "$@" > $log 2>&1
  else
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $PORT bench.py --gpus $n --steps $STEPS --warmup $WARMUP "$@" > $log 2>&1
  fi
  local rc=$?
  local line
  line=$(grep '^{"metric"' $log | tail -n 1)
  if [ $rc -eq 0 ] && [ -n "$line" ]; then
    echo "$line" >> $RAW
    echo "ok   $tag: $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], "ms", d["value"], "tok/s")')"
  else
    echo "{\"failed\": \"$tag\", \"rc\": $rc}" >> $RAW
    echo "FAIL $tag rc=$rc (see $log)"
    case $rc in 124|137|134|139) echo "stopping: hang or crash"; exit $rc ;; esac
  fi
}
for par in dp tp pp; do
  for n in 1 2 4 8; do
    run ${par}${n} $n --parallel $par
  done
done
run gpt2medium_dp4tp2 8 --model gpt2-medium --parallel dp --tp 2
python scripts/scaling_report.py $RAW --json $OUT/scaling.json --md $OUT/scaling.md
