set -o pipefail
# r05a: where the captured decoder step's time goes, kernel family by family, in the chain (decode alone)
O=gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/decode_chain_costs.py --rows 24 15 > $O/chain.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/step.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python scripts/decode_step_time.py --rows 24 --reps 1 > $O/kt.log 2>&1 || exit $?
cat $O/chain.log $O/step.log
