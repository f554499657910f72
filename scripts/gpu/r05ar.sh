# k_layernorm_mx with 32-row workgroups (scale lines through LDS, 8 rows per wave in flight) against the r05aq kernel,
# the 2-rows-in-flight probe (u1) and the no-scale-store probe; MX / fp8-encoder tests; config 5 bench
set -o pipefail
O=$PWD/gpurun_out/r05ar; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8_encoder.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  echo "== r05aq $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py --lib scripts/exp/libtwhip_lnq_r05aq.so || exit $?
  echo "== new $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py || exit $?
  echo "== u1 $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py --lib scripts/exp/libtwhip_lnq_u1.so || exit $?
  echo "== noscale $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py --lib scripts/exp/libtwhip_lnq_noscale.so || exit $?
done > $O/ln.txt 2>&1 || { tail -20 $O/ln.txt; exit 1; }
grep -v amdgpu.ids $O/ln.txt
timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
grep '^{' $O/c5.log | tail -1 > $O/c5.json
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'], d['parity'], d['roofline']['achieved'], d['roofline']['frac'])"
