set -o pipefail
# new front-end kernels (k8 log-mel, implicit conv2), long-form input, condition_on_prev_tokens, beam word timestamps,
# then the e2e suites the decode-pass changes touch
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_longform.py -x -v -s -k "logmel or conv2 or long or masked" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/new.log 2>&1 || { tail -40 $O/new.log; exit 1; }
grep -E "PASS|FAIL|exact|differs" $O/new.log | tail -30
timeout -k 10 600 python -u -m pytest tests/test_gpu_word.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/word.log 2>&1 || { tail -40 $O/word.log; exit 1; }
grep -E "PASS|FAIL|beam|differs" $O/word.log | tail -20
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_beam.py tests/test_gpu_fallback.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/e2e.log 2>&1 || { tail -40 $O/e2e.log; exit 1; }
tail -2 $O/e2e.log
