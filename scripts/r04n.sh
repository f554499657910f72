set -o pipefail
# round-4 final evidence, call 2: config 5 (rocprof, PMC, bench with fp8 parity)
BENCH_ARGS="--config c5" bash scripts/gpu_round.sh r04n_c5 1 || exit $?
echo final-c5-done
