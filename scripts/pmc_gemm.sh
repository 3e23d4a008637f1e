#!/bin/bash
# Two PMC passes (each its own rocprofv3 run, counter budget per pass respected) over the layer-GEMM
# epilogue micro: bash scripts/pmc_gemm.sh  -> gpurun_out/pmc1, gpurun_out/pmc2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/pmc1 -o pmc --output-format csv -- python benchmarks/gemm_epi_micro.py > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/pmc2 -o pmc --output-format csv -- python benchmarks/gemm_epi_micro.py > gpurun_out/pmc2.log 2>&1
