# k_gemm_mx slimmed to 182 VGPRs (buffer descriptors, packed W scales, lane-offset fragment addresses, two W-fragment
# passes) as the MX GEMM beside config 5's decode (TW_MX_BESIDE=1) vs k_gemm_8p_mx (8): MX tests, the kernels alone,
# then config 5 interleaved
set -o pipefail
O=$PWD/gpurun_out/r05ba; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8_encoder.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 1,8 --m 96000 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep '^{' $O/ab.txt
for i in 1 2; do
  for v in 8 1; do
    TW_MX_BESIDE=$v timeout -k 10 400 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
    echo "c5 mx_beside=$v $(grep '^{' $O/c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['parity'], d['roofline']['achieved'])")"
  done
done
