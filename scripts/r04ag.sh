set -o pipefail
# configs 5 and 3 at HEAD (after the round-4 close fixes): the fp8 64-window line and the C3 one-GPU share
O=gpurun_out/r04ag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
grep '^{' $O/c5.log | tail -1 > $O/c5.json
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
grep '^{' $O/c3.log | tail -1 > $O/c3.json
python -c "
import json
for n in ('c5','c3'):
    d=json.load(open('$O/'+n+'.json')); print(n, d['ms_per_step'], d['value'], d.get('parity'), d['config'].get('c3_share'))"
