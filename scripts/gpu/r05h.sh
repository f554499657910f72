set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/decode_step_time.py --rows 15 24 64 --check-every 8 --graph-steps 1 > $O/step.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
cat $O/step.log; grep '^{' $O/bench.log | tail -1 | cut -c1-400
