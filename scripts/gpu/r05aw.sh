# k_gemv_q for <= 16-row decode passes (tw_gemv_set_variant 2, TW_DEC_ALONE_GEMV=2): decode step alone at 15 rows,
# then config 3's 8-GPU share (15 windows, RCCL path forced), interleaved against the shipped choice (1)
set -o pipefail
O=$PWD/gpurun_out/r05aw; mkdir -p $O
for g in 1 2; do
  echo "== gemv $g"; TW_DEC_ALONE_GEMV=$g timeout -k 10 300 python -u scripts/decode_step_time.py --rows 15 24 --reps 3 2>&1 | grep '^{' || exit 1
done
for i in 1 2; do
  for g in 1 2; do
    TW_DEC_ALONE_GEMV=$g timeout -k 10 300 python -u bench.py --config c3 --c3-share 8 --force-collective --steps 5 --warmup 2 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
    echo "c3share gemv=$g $(grep '^{' $O/c3.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d.get('parity'))")"
  done
done
