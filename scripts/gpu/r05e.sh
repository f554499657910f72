set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/decode_step_time.py --rows 24 --check-every 8 --graph-steps 1 8 --slope 1 > $O/step.log 2>&1 || exit $?
cat $O/step.log
