set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/decode_step.log 2>&1 || exit $?
grep '^{' $O/decode_step.log
for r in 1 2; do for a in 16 32; do
  TW_ENC_ATTN=$a timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_attn${a}_$r.log 2>&1 || exit $?
  echo "attn=$a round=$r $(grep -o '"ms_per_step": [0-9.]*' $O/bench_attn${a}_$r.log)"
done; done
timeout -k 10 600 python -u bench.py --config c3 --c3-share 8 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c3s8.log 2>&1 || exit $?
echo "c3 share8 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c3s8.log)"
timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped.log 2>&1 || exit $?
tail -1 $O/as_shipped.log
