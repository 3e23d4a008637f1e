# A/B: deferred optimizer on/off, 3 runs each (bench.py, no profiler)
set -e
for rep in 1 2 3; do
  for d in true false; do
    r=$(timeout -k 10 300 python bench.py --steps 60 --warmup 5 --set defer_optimizer=$d 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])")
    echo "defer=$d $r"
  done
done
