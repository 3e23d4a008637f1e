#!/bin/bash
# Whole-step hardware counters of bench.py, one rocprofv3 --pmc pass per counter group (the
# per-pass slot budget: <= 8 SQ, <= 4 TCC, FETCH_SIZE and WRITE_SIZE in separate passes):
#   bash scripts/pmc_step.sh  -> gpurun_out/pmc_step{1,2,3}/ ; summarise with scripts/pmc_summary.py
#   BENCH_ARGS="--model ref --set dtype=fp32" PMC_TAG=fp32 bash scripts/pmc_step.sh -> gpurun_out/pmc_fp32{1,2,3}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
TAG="${PMC_TAG:-step}"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d gpurun_out/pmc_$TAG$i -o pmc --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --ref32 off ${BENCH_ARGS:-} > gpurun_out/pmc_$TAG$i.log 2>&1 || exit $?
done
