set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_c3_c4.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -3 $O/gputest.txt
timeout -k 10 300 python -u bench.py --force-collective --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_forced.log 2>&1 || exit $?
grep '^{' $O/c2_forced.log | tail -1 > $O/c2_forced.json
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_full.log 2>&1 || exit $?
grep '^{' $O/c3_full.log | tail -1 > $O/c3_full.json
timeout -k 10 300 python -u bench.py --config c3 --c3-share 8 --force-collective --steps 5 --warmup 2 --no-cpu-baseline > $O/c3_share8.log 2>&1 || exit $?
grep '^{' $O/c3_share8.log | tail -1 > $O/c3_share8.json
timeout -k 10 300 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped.log 2>&1 || exit $?
grep '^{' $O/as_shipped.log | tail -1 > $O/as_shipped_turbo.json
timeout -k 10 400 python -u scripts/exp/as_shipped_rtf.py --model large-v3 > $O/as_shipped_v3.log 2>&1 || exit $?
grep '^{' $O/as_shipped_v3.log | tail -1 > $O/as_shipped_large_v3.json
for f in c2_forced c3_full c3_share8; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['ms_per_step'], d['value'], d['config'].get('collectives'), d.get('parity'))"; done
cat $O/as_shipped_turbo.json $O/as_shipped_large_v3.json
