set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/decode_kernel_chains.py --rows 24 > $O/chains.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/decode_chain_costs.py --rows 24 --variants 0 1 --families 0 > $O/chain.log 2>&1 || exit $?
cat $O/chains.log $O/chain.log
