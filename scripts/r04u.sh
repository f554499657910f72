set -o pipefail
# same-box A/B: HEAD vs the end of round 3 (fcb0194), interleaved config 2 bench
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
run() {  # run NAME DIR
  (cd $2 && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/$1.log 2>&1 || exit $?
  echo "$1 $(grep '^{' $O/$1.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["parity"])')"
}
for r in 1 2 3; do
  run head_$r .
  run r03end_$r _r03end
done
echo ab-done
