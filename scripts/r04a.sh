set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_beam.py tests/test_gpu_turbo.py tests/test_gpu_c3_c4.py -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit $?
tail -c 3000 $O/bench.log
TW_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench2.log 2>&1 || exit $?
tail -c 1500 $O/bench2.log
