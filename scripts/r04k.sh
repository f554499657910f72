set -o pipefail
# combined call options (word timestamps with long-form / conditioning / fallback; fallback with beams) + the suites
# whose code paths they share
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_combos.py tests/test_gpu_word.py tests/test_gpu_longform.py tests/test_gpu_fallback.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|exact|differs|same transcript" $O/tests.log | tail -60
