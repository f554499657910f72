set -o pipefail
# proj_out capped at 128 registers (HEAD) vs uncapped (_base tree): GEMV tests, interleaved config 2 bench, decode alone
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemv" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # run NAME DIR
  (cd $2 && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/$1.log 2>&1 || exit $?
  echo "$1 $(grep '^{' $O/$1.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["parity"])')"
}
for r in 1 2 3; do
  run cap_$r .
  run base_$r _base
done
timeout -k 10 600 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/dec.log 2>&1 || exit $?
grep '^{' $O/dec.log
echo ab-done
