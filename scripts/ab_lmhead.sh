set -e
for cfg in "7 side" "7 main" "3 side" "3 main"; do
  set -- $cfg
  echo "DTC_GEMM256=$1 DTC_LMHEAD_WGRAD=$2"
  DTC_GEMM256=$1 DTC_LMHEAD_WGRAD=$2 timeout -k 10 300 python bench.py --steps 40 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])"
done
