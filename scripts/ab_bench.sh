#!/bin/bash
# Interleaved A/B of whole-step time: bench.py under each variant, ROUNDS rounds.
#   ROUNDS=3 bash scripts/ab_bench.sh "DTC_X=0" "DTC_X=1|--set defer_optimizer=true" ...
# A variant is "ENV=... ENV=...|bench args" (either part may be empty).  Prints one line per run
# (variant, ms/step); per-run logs under gpurun_out/ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
ROUNDS=${ROUNDS:-3}
STEPS=${STEPS:-50}
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=${v%%|*}
    args=""
    [[ "$v" == *"|"* ]] && args=${v#*|}
    log=gpurun_out/ab/r${r}_v${i}.log
    # shellcheck disable=SC2086
    env $envs timeout -k 10 120 python bench.py --steps "$STEPS" --warmup 5 --ref32 off $args > "$log" 2>&1 || { echo "FAIL variant [$v] rc=$?"; tail -5 "$log"; exit 1; }
    ms=$(grep -o '"ms_per_step": [0-9.]*' "$log" | awk '{print $2}')
    echo "round $r variant [$v] ms_per_step $ms" | tee -a gpurun_out/ab/summary.log
  done
done
