set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for cfg in "TW_WAIT=sync" "TW_WAIT=poll"; do
  for fc in "" "--force-collective"; do
    env $cfg timeout -k 10 300 python -u bench.py $fc --steps 10 --warmup 2 --no-cpu-baseline > $O/b.log 2>&1 || exit $?
    echo "$cfg $fc $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['parity'])")"
  done
done
done
