set -o pipefail
# r05b: k_gemv_q (one column group per wave, K-slice in one batch) vs k_gemv_pc in the captured step
O=gpurun_out/r05b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/decode_chain_costs.py --rows 24 15 64 --variants 0 1 0 1 --families 0 > $O/chain.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python scripts/decode_chain_costs.py --rows 24 --variants 1 --families 0 --reps 20 > $O/kt.log 2>&1 || exit $?
cat $O/chain.log
