set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/decode_chain_costs.py --rows 15 24 64 --families 0 --variants 0 1 --wide-kw 1 2 4 --reps 100 > $O/c.log 2>&1 || exit $?
cat $O/c.log
