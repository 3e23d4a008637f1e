# A/B of TrainConfig overrides: bash scripts/ab_set.sh "KEY=V1 KEY=V2 ..." [reps]  (one --set per setting;
# "-" = defaults); prints every rep's ms/step and the min per setting, settings interleaved
VALS=$1; REPS=${2:-3}
declare -A res
for rep in $(seq $REPS); do
  for v in $VALS; do
    if [ "$v" = "-" ]; then a=""; else a="--set $v"; fi
    r=$(timeout -k 10 300 python bench.py --steps 60 --warmup 5 --ref32 off $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])") || exit 1
    res[$v]="${res[$v]} $r"
  done
done
for v in $VALS; do
  echo "$v: ${res[$v]} -> min $(echo ${res[$v]} | tr ' ' '\n' | sort -n | head -1)"
done
