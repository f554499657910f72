# the bench with the slot-parity warmup fix: HEAD at 20/5 and at the defaults (5/2), k_gemv_q alone on and off
set -o pipefail
O=$PWD/gpurun_out/r05aj; mkdir -p $O
run() {  # run LABEL DIR STEPS WARMUP [ENV...]
  local label=$1 dir=$2 k=$3 w=$4; shift 4
  (cd $dir && env "$@" timeout -k 10 300 python -u bench.py --steps $k --warmup $w --no-cpu-baseline > $O/b.log 2>&1) || exit $?
  echo "$label $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
}
for i in 1 2 3; do
  run head_20_5 . 20 5 TW_X=0
  run head_gemv0_20_5 . 20 5 TW_DEC_ALONE_GEMV=0
  run head_5_2 . 5 2 TW_X=0
  run r04_20_5 _ab_r04 20 5 TW_X=0
done
