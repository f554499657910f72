# the encoder GEMM queued beside a decode: k_gemm_big on all CUs (shipped) vs the persistent k_gemm_8pp on 224 / 192
# CUs (the rest free for the decoder), 20-step bench, interleaved
set -o pipefail
O=gpurun_out/r05af; mkdir -p $O
for i in 1 2; do
for e in "TW_GEMM_BESIDE=1" "TW_GEMM_BESIDE=6 TW_GEMM_BESIDE_CUS=224" "TW_GEMM_BESIDE=6 TW_GEMM_BESIDE_CUS=192" "TW_GEMM_BESIDE=6 TW_GEMM_BESIDE_CUS=240"; do
  env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit $?
  echo "$e $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
done
done
