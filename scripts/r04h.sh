set -o pipefail
# round-4 evidence at HEAD: the new front-end kernels' tests first, then the whole GPU suite + config 2 round
# (rocprof, PMC, bench); config 5's round is a second call (scripts/gpu_round.sh r04h_c5 1 with --config c5)
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "logmel or conv2" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04h/fe_tests.log 2>&1 || { tail -30 gpurun_out/r04h/fe_tests.log; exit 1; }
tail -1 gpurun_out/r04h/fe_tests.log
bash scripts/gpu_round.sh r04h || exit $?
