# A/B: minimum tile count for the 256^2 kernel (fwd + ordinary dgrad)
set -e
for mt in 512 96 64; do
  echo "DTC_BIG_MIN_TILES=$mt"
  DTC_BIG_MIN_TILES=$mt timeout -k 10 300 python bench.py --steps 40 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])"
done
DTC_BIG_MIN_TILES=64 timeout -k 10 300 python benchmarks/gemm_bench.py > gpurun_out/gemmb_big64.log 2>&1
