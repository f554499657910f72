# same-box bisection of the round-5 bench regression (r05ah: HEAD 90.8 vs round-4 88.0 ms/step): the round-5 commits
# that touched the decode loop / GEMV kernels, built in git worktrees, plus HEAD with the decode-loop env knobs
set -o pipefail
O=$PWD/gpurun_out/r05ai; mkdir -p $O
run() {  # run LABEL DIR [ENV...]
  local label=$1 dir=$2; shift 2
  (cd $dir && env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1) || exit $?
  echo "$label $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
}
for i in 1 2 3; do
  run head . TW_X=0
  run r04 _ab_r04 TW_X=0
  run c63a7a0c _ab_63a7a0c TW_X=0
  run c9100578 _ab_9100578 TW_X=0
  run c23a5371 _ab_23a5371 TW_X=0
  run c36fc1e1 _ab_36fc1e1 TW_X=0
  run head_sync . TW_WAIT=sync
  run head_gemv0 . TW_DEC_ALONE_GEMV=0
done
