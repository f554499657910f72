set -e
mkdir -p gpurun_out/lnst
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "stats or lnst or gemv" -p no:cacheprovider > gpurun_out/lnst/kern.log 2>&1 || { tail -30 gpurun_out/lnst/kern.log; exit 1; }
tail -2 gpurun_out/lnst/kern.log
TW_DEC_LNSTATS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_configs.py tests/test_gpu_beam.py tests/test_gpu_word.py -x -q -p no:cacheprovider > gpurun_out/lnst/e2e.log 2>&1 || { tail -30 gpurun_out/lnst/e2e.log; exit 1; }
tail -2 gpurun_out/lnst/e2e.log
bash scripts/exp/ab_env.sh "TW_DEC_LNSTATS=0" "TW_DEC_LNSTATS=1" 3
