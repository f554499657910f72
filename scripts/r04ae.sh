set -o pipefail
# round-4 close at HEAD (after prompt_ids): suite + kernel trace + PMC passes + bench (gpu_round.sh), smoke(), and the
# bench as the driver runs it (20 steps, 5 warm-up)
bash scripts/gpu_round.sh r04ae || exit 1
O=gpurun_out/r04ae
timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
grep '^{' $O/bench20.log | tail -1 > $O/bench20.json
python -c "import json; d=json.load(open('$O/bench20.json')); print(d['ms_per_step'], d['value'], d['parity'], d['roofline']['frac'])"
