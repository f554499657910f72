set -o pipefail
# round-4 extras at HEAD: free-running decode (EOS allowed) and the self-spawning 2-rank launcher (gloo rehearsal
# on the one GPU: both ranks share it, so the value is a control-path check, not a scaling number)
O=gpurun_out/r04ai; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --eos --steps 5 --warmup 2 --no-cpu-baseline > $O/eos.log 2>&1 || exit $?
grep '^{' $O/eos.log | tail -1 > $O/bench_eos.json
TW_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/gpus2.log 2>&1 || exit $?
grep '^{' $O/gpus2.log | tail -1 > $O/bench_gpus2_gloo_spawn.json
python -c "import json; d=json.load(open('$O/bench_eos.json')); print('eos', d['ms_per_step'], d['value']); d=json.load(open('$O/bench_gpus2_gloo_spawn.json')); print('gpus2', d['n_gpus'], d['ms_per_step'], d['value'])"
