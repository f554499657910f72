# C5 bench against the round-5 pass/wait/GEMM knobs (one box)
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
for e in "TW_X=0" "TW_DEC_ALONE_GEMV=0" "TW_WAIT=sync" "TW_GEMM_ALONE=5" "TW_GRAPH_STEPS_ALONE=1" "TW_X=0"; do
  env $e timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.log 2>&1 || exit $?
  echo "$e $(grep '^{' $O/c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
done
