set -o pipefail
# same-box A/B: HEAD vs the r04e tree (commit 54182ae, 90.7 ms per step on its box), interleaved, config 2 bench
O=gpurun_out/r04p; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/head_$r.log 2>&1 || exit $?
  echo "head_$r $(grep '^{' $O/head_$r.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  (cd _old_r04e && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/old_$r.log 2>&1 || exit $?
  echo "r04e_$r $(grep '^{' $O/old_$r.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
echo ab-done
