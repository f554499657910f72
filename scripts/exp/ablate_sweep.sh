# Timing-only ablation sweep of the bench step (outputs are wrong with any stage skipped):
#   bash scripts/exp/ablate_sweep.sh "ln cross self eattn eln egemm"
set -e
for ab in none $1; do
  a=$ab; [ "$ab" = none ] && a=""
  TW_ABLATE=$a timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abl.log 2>&1
  echo "ablate=$ab $(tail -1 gpurun_out/abl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
