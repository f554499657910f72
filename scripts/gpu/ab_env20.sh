# A/B of environment settings on the 20-step bench (the driver's length): bash scripts/gpu/ab_env20.sh "VAR=a" "VAR=b" [reps]
set -o pipefail
reps=${3:-2}
mkdir -p gpurun_out
for i in $(seq 1 $reps); do
  for e in "$1" "$2"; do
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
    echo "$e $(grep '^{' gpurun_out/ab.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
  done
done
