set -e
for rep in 1 2; do
  for s in 0 1; do
    r=$(DTC_SIDE_INTERLEAVE=$s timeout -k 10 300 python bench.py --steps 60 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])")
    echo "interleave=$s $r"
  done
done
