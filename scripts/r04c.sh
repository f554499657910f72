set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_mx.py tests/test_gpu_fp8_encoder.py tests/test_gpu_word.py tests/test_gpu_c3_c4.py -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/decode_step_time.py > $O/decode_step.log 2>&1 || exit $?
cat $O/decode_step.log | grep '^{'
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"parity": [a-z]*\|"positions_checked": [0-9]*' $O/bench.log
timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"parity": [a-z]*\|"positions_checked": [0-9]*' $O/bench_c5.log
timeout -k 10 600 python -u bench.py --config c3 --c3-share 8 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c3s8.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench_c3s8.log
timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped.log 2>&1 || exit $?
tail -3 $O/as_shipped.log
