# Generic A/B: bash scripts/ab_env.sh VAR "v1 v2 ..." [reps]; prints min/median ms per setting
VAR=$1; VALS=$2; REPS=${3:-4}
declare -A res
for rep in $(seq $REPS); do
  for v in $VALS; do
    r=$(env $VAR=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 --ref32 off 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])") || exit 1
    res[$v]="${res[$v]} $r"
  done
done
for v in $VALS; do
  echo "$VAR=$v: ${res[$v]} -> min $(echo ${res[$v]} | tr ' ' '\n' | sort -n | head -1)"
done
