set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemv or resid" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u scripts/decode_step_time.py --rows 24 64 > $O/decode_step.log 2>&1 || exit $?
grep '^{' $O/decode_step.log
timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped.log 2>&1 || exit $?
tail -1 $O/as_shipped.log
timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"parity": [a-z]*' $O/bench_c5.log
