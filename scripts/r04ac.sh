set -o pipefail
O=gpurun_out/r04ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_audio.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/audio.log 2>&1 || { tail -40 $O/audio.log; exit 1; }
grep -E "PASS|FAIL" $O/audio.log | tail -20
