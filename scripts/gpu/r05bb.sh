# config 5 with the MX kernel by shape (9: k_gemm_mx for q/k/v, k_gemm_8p_mx for the rest; alone and beside the decode)
# vs k_gemm_8p_mx everywhere (0 / 8), interleaved; the shape A/B alone first
set -o pipefail
O=$PWD/gpurun_out/r05bb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 8 9; do
    TW_MX_BESIDE=$v TW_MX_ALONE=$v timeout -k 10 400 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
    echo "c5 mx=$v $(grep '^{' $O/c5.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['parity'], d['roofline']['achieved'])")"
  done
done
