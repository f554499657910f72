set -o pipefail
# round-4 final evidence, call 1: the whole GPU suite + config 2 (rocprof kernel stats, PMC traffic / MFMA, bench)
bash scripts/gpu_round.sh r04m || exit $?
echo final-c2-done
