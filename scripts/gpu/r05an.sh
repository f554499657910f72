# k_gemm_8p_mx with the residual-line prefetch (8) vs without (9), same build, interleaved; MX GPU tests first
set -o pipefail
O=$PWD/gpurun_out/r05an; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/mx_tests.log 2>&1 || { tail -30 $O/mx_tests.log; exit 1; }
tail -2 $O/mx_tests.log
timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8,9 --reps 7 --m 96000,36000 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep '^{' $O/ab.txt
