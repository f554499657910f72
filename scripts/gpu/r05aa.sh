# C5 bench: default vs the decode pass's k_gemv_pc alone (TW_DEC_ALONE_GEMV=0), 10 steps, 3 interleaved pairs
set -o pipefail
O=gpurun_out/r05aa; mkdir -p $O
for i in 1 2 3; do
for e in "TW_X=0" "TW_DEC_ALONE_GEMV=0"; do
  env $e timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5.log 2>&1 || exit $?
  echo "$e $(grep '^{' $O/c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
done
done
