set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -3 gpurun_out/sk_tests.log
GEMM_BENCH_NO_MX=1 timeout -k 10 300 python -u scripts/gemm_bench.py --rounds 5 > gpurun_out/sk_bench.log 2>&1; rc=$?
cat gpurun_out/sk_bench.log; exit $rc
