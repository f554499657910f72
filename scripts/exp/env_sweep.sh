# One bench line per environment setting: bash scripts/exp/env_sweep.sh "A=1" "A=2 B=3" ...
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sweep.log 2>&1 || { echo "$e FAILED"; tail -5 gpurun_out/sweep.log; exit 1; }
  echo "$e $(tail -1 gpurun_out/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])")"
done
