# k_gemm_8p_mx RESID epilogue with addends loaded ahead + straight-line interior path: MX GPU tests, the MX GEMM
# shapes against the previous build (scripts/exp/libtwhip_pre_mxresid.so), interleaved, then config 5's bench
set -o pipefail
O=$PWD/gpurun_out/r05am; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/mx_tests.log 2>&1 || { tail -30 $O/mx_tests.log; exit 1; }
tail -2 $O/mx_tests.log
for i in 1 2; do
  echo "== old $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000,36000 --lib scripts/exp/libtwhip_pre_mxresid.so || exit $?
  echo "== new $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000,36000 || exit $?
done > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
grep '^{' $O/c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], d['parity'], d['roofline']['achieved'], d['roofline']['frac'])"
