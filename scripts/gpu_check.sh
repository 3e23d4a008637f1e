#!/bin/bash
# GPU-box validation: each GPU step under its own timeout; stop at the first crash/timeout
# (exit codes other than 0 = pass / 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc" | tee -a gpurun_out/summary.log; exit $rc; fi
  return 0
}
STEPS="${STEPS:-kernels engine smoke bench}"
for s in $STEPS; do
  case $s in
    kernels) run kernels 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -rf ;;
    engine)  run engine 600 python -m pytest tests/test_engine_gpu.py -q -m gpu -rf ;;
    gpu)     run gpu 900 python -m pytest tests -q -m gpu -rf ;;
    dist)    run dist 900 python -m pytest tests/test_dist_gpu.py -q -m gpu -rf ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 600 python bench.py --steps 30 --warmup 5 ;;  # (+ the ref_fp32 point)
    benchng) run benchng 600 python bench.py --steps 20 --warmup 3 --no_graph ;;
    gemmb)   run gemmb 600 python benchmarks/gemm_bench.py --json gpurun_out/gemm_bench.json ;;
    prof)    run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 --ref32 off ;;
  esac
done
echo ALLDONE | tee -a gpurun_out/summary.log
