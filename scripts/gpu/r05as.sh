# GELU-MX epilogue block absmax by DPP quad permutes: MX / fp8-encoder tests, the MX shapes against the previous build
# (scripts/exp/libtwhip_pre_gelumx.so), config 5 bench
set -o pipefail
O=$PWD/gpurun_out/r05as; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8_encoder.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  echo "== old $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000 --lib scripts/exp/libtwhip_pre_gelumx.so || exit $?
  echo "== new $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000 || exit $?
done > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
grep '^{' $O/c5.log | tail -1 > $O/c5.json
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'], d['parity'], d['roofline']['achieved'], d['roofline']['frac'])"
