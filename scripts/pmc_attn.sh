#!/bin/bash
# Hardware counters of the attention kernels at the reference shape (benchmarks/attn_micro.py),
# one rocprofv3 --pmc pass per counter group (<= 8 SQ counters per pass):
#   bash scripts/pmc_attn.sh -> gpurun_out/pmc_attn{1,2}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_attn$i -o pmc --output-format csv -- \
    python benchmarks/attn_micro.py > gpurun_out/pmc_attn$i.log 2>&1 || exit $?  # ATTN_SHAPE=medium: T 1024 / hd 64
done
