set -o pipefail
# round-4 final evidence after the decoder register fixes: the whole GPU suite + config 2 (kernel trace, PMC, bench)
bash scripts/gpu_round.sh r04t || exit $?
echo final-c2-done
