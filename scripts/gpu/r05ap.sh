# k_layernorm_mx sized to the row (NC template) with gamma / beta loaded beside it and the block absmax by DPP: MX and
# fp8-encoder GPU tests, then the LayerNorm against the previous build (bit-identical outputs expected), interleaved
set -o pipefail
O=$PWD/gpurun_out/r05ap; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8_encoder.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  echo "== old $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py --lib scripts/exp/libtwhip_pre_mxresid.so || exit $?
  echo "== new $i"; timeout -k 10 120 python -u scripts/exp/ln_mx_time.py || exit $?
done > $O/ln.txt 2>&1 || { tail -20 $O/ln.txt; exit 1; }
grep -v amdgpu.ids $O/ln.txt
