#!/bin/bash
# gemm8p with contiguous A chunks: numerics, lm_head A/B, PMC on the MN-major wgrad
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or lmhead or ce_" > gpurun_out/r3_g8pb_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 gpurun_out/r3_g8pb_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  DTC_GEMM8P=$v timeout -k 10 300 python benchmarks/gemm_bench.py --model gpt2-small --reps 30 --only lm_head --no-ref > gpurun_out/r3_g8pb_bench_$v.log 2>&1 || exit $?
  echo "== DTC_GEMM8P=$v"; grep -v amdgpu.ids gpurun_out/r3_g8pb_bench_$v.log
done
for P in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum FETCH_SIZE"; do
  i=$((${i:-0} + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmc_g8p$i -o pmc --output-format csv -- python benchmarks/gemm_bench.py --model gpt2-small --reps 5 --only "wgrad lm_head,dgrad lm_head" --no-ref > gpurun_out/pmc_g8p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -3 gpurun_out/pmc_g8p$i.log; exit 1; }
done
echo pmc done
