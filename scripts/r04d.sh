set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 900 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/decode_step.log 2>&1 || exit $?
grep '^{' $O/decode_step.log
for cfg in "1 1 32" "0 1 32" "1 0 32" "0 0 32" "0 0 16"; do
  set -- $cfg
  TW_FUSE_SELF=$1 TW_FUSE_CROSS=$2 TW_ENC_ATTN=$3 timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$1$2_$3.log 2>&1 || exit $?
  echo "self=$1 cross=$2 attn=$3 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$1$2_$3.log)"
done
