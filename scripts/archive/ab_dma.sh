# A/B of the DMA-pipelined layer GEMM kernel: numerics at each setting, then step time + per-GEMM timings
set -e
for cfg in "0 2" "1 2" "3 2" "3 3"; do
  set -- $cfg
  echo "=== DTC_GEMM_DMA=$1 DTC_DMA_STAGES128=$2"
  DTC_GEMM_DMA=$1 DTC_DMA_STAGES128=$2 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" 2>&1 | tail -1
  DTC_GEMM_DMA=$1 DTC_DMA_STAGES128=$2 timeout -k 10 300 python bench.py --steps 40 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms/step', d['ms_per_step'])"
  DTC_GEMM_DMA=$1 DTC_DMA_STAGES128=$2 timeout -k 10 300 python benchmarks/gemm_bench.py 2>/dev/null | grep -v lm_head | grep -v attn | grep -v colsum
done
