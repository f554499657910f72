# MX LayerNorm: what the scale-byte stores cost (probe build without them, scripts/exp/libtwhip_lnq_noscale.so) against
# the shipped kernel, then config 5's bench with the new LayerNorm (20 steps, 5 warm-up)
set -o pipefail
O=$PWD/gpurun_out/r05aq; mkdir -p $O
for i in 1 2; do
  echo "== noscale $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py --lib scripts/exp/libtwhip_lnq_noscale.so || exit $?
  echo "== new $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py || exit $?
done > $O/ln.txt 2>&1 || { tail -20 $O/ln.txt; exit 1; }
grep -v amdgpu.ids $O/ln.txt
timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
grep '^{' $O/c5.log | tail -1 > $O/c5.json
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'], d['parity'], d['roofline']['achieved'], d['roofline']['frac'])"
