# k_gemm_8p_mx without hipcc's per-phase vmcnt(0) drains: MX GPU tests, the MX shapes against the pre-fix build
# (scripts/exp/libtwhip_pre_mxresid.so), then config 5's round profile + bench (gpu_round.sh, tests skipped)
set -o pipefail
O=$PWD/gpurun_out/r05ao; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/mx_tests.log 2>&1 || { tail -30 $O/mx_tests.log; exit 1; }
tail -2 $O/mx_tests.log
for i in 1 2; do
  echo "== old $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000,36000 --lib scripts/exp/libtwhip_pre_mxresid.so || exit $?
  echo "== new $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000,36000 || exit $?
done > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
BENCH_ARGS="--config c5" bash scripts/gpu_round.sh r05ao_c5 1
