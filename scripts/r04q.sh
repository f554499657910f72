set -o pipefail
# same-box bisection of the config-2 step between r04e (54182ae) and HEAD, interleaved
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
run() {  # run NAME DIR
  (cd $2 && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/$1.log 2>&1 || exit $?
  echo "$1 $(grep '^{' $O/$1.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for r in 1 2; do
  run r04e_$r _old_r04e
  run f69a94e_$r _old_f69a94e
  run 434daa8_$r _old_434daa8
  run head_$r .
done
echo ab-done
