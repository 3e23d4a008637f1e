# A/B of whole env settings: bash scripts/ab_multi.sh REPS "VAR=a VAR2=b" "VAR=c" ...  ("-" = no extra env)
# prints every run's ms/step and the min per setting (runs interleaved to spread box drift)
REPS=$1; shift
declare -A res
for rep in $(seq $REPS); do
  for cfg in "$@"; do
    envs=""; [ "$cfg" != "-" ] && envs="$cfg"
    r=$(env $envs timeout -k 10 300 python bench.py --steps 60 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'])") || exit 1
    res[$cfg]="${res[$cfg]} $r"
  done
done
for cfg in "$@"; do
  echo "[$cfg]: ${res[$cfg]} -> min $(echo ${res[$cfg]} | tr ' ' '\n' | sort -n | head -1)"
done
