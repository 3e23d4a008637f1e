#!/bin/bash
# SURVEY §6.4 oracle-agreement criterion: 5000 timed steps of the reference DP config in bf16 (the
# default) and in exact fp32 (the reference's precision, our fp32 MFMA kernels), same data and init.
#   -> gpurun_out/parity/{bf16,fp32}/log.csv ; report: python scripts/parity_report.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/parity
for dt in bf16 fp32; do
  timeout -k 10 500 python main.py --train_config_path configs/train_config_dp.yaml --log_every 500 --dtype $dt \
      --output_dir gpurun_out/parity/$dt > gpurun_out/parity/main_$dt.log 2>&1 || exit $?
  tail -n 3 gpurun_out/parity/main_$dt.log
done
