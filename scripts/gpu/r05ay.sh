# HEAD check after the bench warmup refactor: config 2 as the driver runs it, and the 5-step default
set -o pipefail
O=$PWD/gpurun_out/r05ay; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
grep '^{' $O/c2.log | tail -1 > $O/c2.json
python -c "import json; d=json.load(open('$O/c2.json')); print('c2', d['value'], d['ms_per_step'], d['parity'], d['warmup_extra_batches'], d['roofline']['frac'], d['cpu_baseline']['value'])"
# config 5: the encoder pump depth beside its 64-row decode (TW_PUMP_AHEAD, default 2), interleaved
for p in 2 1 3 2; do
  TW_PUMP_AHEAD=$p timeout -k 10 400 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
  echo "c5 pump=$p $(grep '^{' $O/c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['parity'])")"
done
