set -o pipefail
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -2 $O/gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
timeout -k 10 400 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/step.log 2>&1 || exit $?
cat $O/step.log
