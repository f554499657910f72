# Interleaved A/B of environment settings on the bench (one line per run):
#   bash scripts/exp/ab_multi.sh REPS STEPS "VAR=a" "VAR=b" ...     ("-" = no extra setting)
set -e
reps=$1; steps=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $reps); do
  for e in "$@"; do
    if [ "$e" = "-" ]; then ev=""; else ev="$e"; fi
    env $ev timeout -k 10 300 python bench.py --steps $steps --warmup ${AB_WARMUP:-2} --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { echo "$e FAILED"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "$e $(tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])")"
  done
done
