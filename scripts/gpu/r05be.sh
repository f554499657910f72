# config 5: the MX LayerNorm's workgroups per CU capped beside the decode (TW_LN_PAD_BESIDE KiB of dynamic LDS, now
# honoured by tw_layernorm_mx as by tw_layernorm) vs uncapped (0, the default), interleaved
set -o pipefail
O=$PWD/gpurun_out/r05be; mkdir -p $O
for i in 1 2; do
  for p in 0 48; do
    TW_LN_PAD_BESIDE=$p timeout -k 10 400 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
    echo "c5 ln_pad=$p $(grep '^{' $O/c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['parity'])")"
  done
done
