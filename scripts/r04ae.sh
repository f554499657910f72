set -o pipefail
# round-4 close at HEAD (after prompt_ids): the whole GPU suite on HEAD, smoke(), and the bench as the driver runs it (20 steps, 5 warm-up)
O=gpurun_out/r04ae; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
grep '^{' $O/bench20.log | tail -1 > $O/bench20.json
python -c "import json; d=json.load(open('$O/bench20.json')); print(d['ms_per_step'], d['value'], d['parity'], d['roofline']['frac'])"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof ok
