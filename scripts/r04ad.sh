set -o pipefail
# prompt_ids on the engine + the long-form / conditioning / combos regressions
O=gpurun_out/r04ad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_prompt.py tests/test_gpu_longform.py tests/test_gpu_combos.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|exact|differs" $O/tests.log | tail -40
