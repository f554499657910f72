# same-box A/B of HEAD against the round-4 final build (_ab_r04, commit 87ba5ae, built in a git worktree), 20-step bench
set -o pipefail
O=$PWD/gpurun_out/r05ah; mkdir -p $O
run() {  # run LABEL DIR [ENV...]
  local label=$1 dir=$2; shift 2
  (cd $dir && env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1) || exit $?
  echo "$label $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
}
for i in 1 2 3; do
  run head . TW_X=0
  run r04 _ab_r04 TW_X=0
done
run head_capi . TW_ENC_OPS=0
run head_gemm5 . TW_GEMM_ALONE=5
