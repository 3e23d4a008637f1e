#!/bin/bash
# Long cross-strategy loss curves on ONE GPU: the reference model, same data and
# canonical init, STEPS timed steps each:
#   dp1 (1 process), tp2 (2 processes, P2P all-reduce kernels; fp32 / bf16 payloads; bf16 + sequence parallel),
#   pp2 (2 processes, 1F1B / zero-bubble, 8 microbatches)
# The 2-process runs share cuda:0 over gloo (RCCL refuses two ranks on one device).
#   -> gpurun_out/curves/{dp,tp,pp}/log.csv ; report: python scripts/cross_strategy_report.py gpurun_out/curves
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=${STEPS:-2000}
OUT=gpurun_out/curves
mkdir -p $OUT
T="timeout -k 10"
$T 400 python main.py --train_config_path configs/train_config_dp.yaml --nproc 1 --steps $STEPS --log_every 250 \
    --output_dir $OUT/dp > $OUT/dp.log 2>&1 || exit $?
tail -n 2 $OUT/dp.log
DTC_DIST_BACKEND=gloo $T 600 python main.py --train_config_path configs/train_config_tp.yaml --nproc 2 --steps $STEPS \
    --log_every 250 --output_dir $OUT/tp --set tp_comm=p2p --set tp_comm_dtype=fp32 --set tp_sequence_parallel=false > $OUT/tp.log 2>&1 || exit $?
tail -n 2 $OUT/tp.log
DTC_DIST_BACKEND=gloo $T 600 python main.py --train_config_path configs/train_config_tp.yaml --nproc 2 --steps $STEPS \
    --log_every 250 --output_dir $OUT/tp_bf16 --set tp_comm=p2p --set tp_comm_dtype=bf16 --set tp_sequence_parallel=false > $OUT/tp_bf16.log 2>&1 || exit $?
tail -n 2 $OUT/tp_bf16.log
DTC_DIST_BACKEND=gloo $T 600 python main.py --train_config_path configs/train_config_tp.yaml --nproc 2 --steps $STEPS \
    --log_every 250 --output_dir $OUT/tp_sp --set tp_comm=p2p --set tp_comm_dtype=bf16 --set tp_sequence_parallel=true \
    > $OUT/tp_sp.log 2>&1 || exit $?
tail -n 2 $OUT/tp_sp.log
DTC_DIST_BACKEND=gloo $T 900 python main.py --train_config_path configs/train_config_pp_1f1b.yaml --nproc 2 --steps $STEPS \
    --log_every 250 --output_dir $OUT/pp --set pp_comm_dtype=fp32 > $OUT/pp.log 2>&1 || exit $?
tail -n 2 $OUT/pp.log
DTC_DIST_BACKEND=gloo $T 900 python main.py --train_config_path configs/train_config_pp_1f1b.yaml --nproc 2 --steps $STEPS \
    --log_every 250 --output_dir $OUT/pp_zb --set pp_schedule=zb --set pp_comm_dtype=fp32 > $OUT/pp_zb.log 2>&1 || exit $?
tail -n 2 $OUT/pp_zb.log
DTC_DIST_BACKEND=gloo $T 900 python main.py --train_config_path configs/train_config_pp_1f1b.yaml --nproc 2 --steps $STEPS \
    --log_every 250 --output_dir $OUT/pp_bf16 --set pp_comm_dtype=bf16 > $OUT/pp_bf16.log 2>&1 || exit $?
tail -n 2 $OUT/pp_bf16.log
