# bench with the warmup completing every (beside/alone, slot) decode graph: defaults (5/2), 20/5, config 5 defaults
set -o pipefail
O=$PWD/gpurun_out/r05ak; mkdir -p $O
run() {  # run LABEL ARGS...
  local label=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/b.log 2>&1 || exit $?
  echo "$label $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'], d['warmup_extra_batches'])")"
}
for i in 1 2; do
  run c2_5_2
  run c2_20_5 --steps 20 --warmup 5
  run c2_6_2 --steps 6 --warmup 2
done
run c5_5_2 --config c5
run c5_20_5 --config c5 --steps 20 --warmup 5
