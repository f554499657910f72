set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/decode_chain_costs.py --rows 24 --families 0 --passlike 1 --reps 50 > $O/c.log 2>&1 || exit $?
cat $O/c.log
