set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_full.log 2>&1 || exit $?
grep '^{' $O/c3_full.log | tail -1 > $O/c3_full.json
timeout -k 10 300 python -u bench.py --config c3 --c3-share 8 --force-collective --steps 5 --warmup 2 --no-cpu-baseline > $O/c3_share8.log 2>&1 || exit $?
grep '^{' $O/c3_share8.log | tail -1 > $O/c3_share8.json
TW_GEMM_ALONE=5 timeout -k 10 300 python -u bench.py --config c3 --c3-share 8 --force-collective --steps 5 --warmup 2 --no-cpu-baseline > $O/c3_share8_8p.log 2>&1 || exit $?
grep '^{' $O/c3_share8_8p.log | tail -1 > $O/c3_share8_8p.json
for f in c3_full c3_share8 c3_share8_8p; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['ms_per_step'], d['value'], d['config'].get('collectives'), d.get('parity'))"; done
