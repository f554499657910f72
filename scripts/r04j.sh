set -o pipefail
# fallback with beams (renormalised beam log-probs, no-speech at the SOT step, the num_beams reset), beam kernels,
# word timestamps with beams
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fallback.py tests/test_gpu_beam.py tests/test_gpu_word.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|window|beam token|differs" $O/tests.log | tail -60
