# split-K factor of the decoder's d_model-wide projections (o_proj, cross o_proj, fc2): 4 (shipped) vs 2 / 8, 20-step bench
set -o pipefail
O=gpurun_out/r05ag; mkdir -p $O
for i in 1 2; do
for e in "TW_DEC_SPLITS=4" "TW_DEC_SPLITS=2" "TW_DEC_SPLITS=8"; do
  env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit $?
  echo "$e $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
done
done
