#!/bin/bash
# round 4, GPU call B: attention counters (both kernel generations), the new step's kernel trace,
# the headline-config oracle test, TP=8 rehearsal (vocab padded per TP degree)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_attn$i -o pmc --output-format csv -- \
    python benchmarks/attn_micro.py > gpurun_out/pmc_attn$i.log 2>&1 || exit $?
done
echo "attention pmc done"
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_b.log 2>&1 || exit $?
tail -n 1 gpurun_out/prof_b.log
$T 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "gpt2_small_step_vs_oracle" -s > gpurun_out/r4_oracle.log 2>&1; rc=$?
grep -E "worst|PASS|FAIL|Error" gpurun_out/r4_oracle.log | head -5; [ $rc -ne 0 ] && exit $rc
DTC_DIST_BACKEND=gloo $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --parallel tp --steps 3 --warmup 2 --set tp_comm=p2p > gpurun_out/r4_tp8_rehearsal.log 2>&1; rc=$?
grep '^{' gpurun_out/r4_tp8_rehearsal.log | tail -n 1; exit $rc
