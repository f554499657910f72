set -o pipefail
# round-4 A/B on one box (config 2 bench, interleaved): HEAD vs the im2col conv2 (TW_CONV2_IM2COL=1), proj_out K-slices
# for decode passes alone (TW_DEC_ALONE_WIDE_KW 1 vs 4), kernel arguments in device memory (HIP_FORCE_DEV_KERNARG)
O=gpurun_out/r04n; mkdir -p $O
export TMPDIR=/tmp
b() {  # b NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$name.log 2>&1 || exit $?
  echo "$name $(grep '^{' $O/bench_$name.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["parity"])')"
}
for r in 1 2; do
  b head_$r TW_AB=0
  b im2col_$r TW_CONV2_IM2COL=1
  b kw1_$r TW_DEC_ALONE_WIDE_KW=1
  b devkernarg_$r HIP_FORCE_DEV_KERNARG=1
done
for v in "kw1 TW_DEC_ALONE_WIDE_KW=1" "kw4 TW_DEC_ALONE_WIDE_KW=4" "devkernarg1 HIP_FORCE_DEV_KERNARG=1"; do
  set -- $v
  env $2 timeout -k 10 600 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/dec_$1.log 2>&1 || exit $?
  echo "dec $1"; grep '^{' $O/dec_$1.log
done
echo ab-done
