set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_capture.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -3 $O/gputest.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python bench.py --config c3 --c3-share 8 --steps 2 --warmup 1 --profile-only > $O/kt.log 2>&1 || exit $?
python scripts/summarize_prof.py $O > $O/summary.txt 2>&1; head -30 $O/summary.txt
