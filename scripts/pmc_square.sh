#!/bin/bash
# Counters of the 256^2 main loop vs hipBLASLt on 4096^3 / 8192^3 (profiles/r6_gemm_square.md):
# L2 hit rate, MFMA busy, LDS activity, clocks.  One rocprofv3 --pmc pass per group, each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
P3="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmcsq_ours$i -o pmc --output-format csv -- \
    benchmarks/bin/gemm_square_micro > gpurun_out/pmcsq_ours$i.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmcsq_hbl$i -o pmc --output-format csv -- \
    python3 benchmarks/hipblaslt_kernel_names.py > gpurun_out/pmcsq_hbl$i.log 2>&1 || exit $?
done
