# config 2: decoder steps per graph replay beside the encoder pump (TW_GRAPH_STEPS_BESIDE) and alone
# (TW_GRAPH_STEPS_ALONE), against the defaults (1, 1), interleaved, 20/5
set -o pipefail
O=$PWD/gpurun_out/r05az; mkdir -p $O
run() {  # run LABEL ENV...
  local label=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$label $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
}
for i in 1 2; do
  run default TW_X=0
  run beside2 TW_GRAPH_STEPS_BESIDE=2
  run beside4 TW_GRAPH_STEPS_BESIDE=4
  run alone4 TW_GRAPH_STEPS_ALONE=4
done
