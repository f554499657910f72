# (1) k_attn_enc5 with its V^T reads issued from asm (no hipcc vmcnt(0) drain before the PV phase) against the previous
# build (scripts/exp/libtwhip_pre_attnvt.so); (2) the GELU-MX epilogue's block absmax by DPP against
# scripts/exp/libtwhip_pre_gelumx.so; attention / MX / fp8-encoder GPU tests; config 2 and config 5 benches
set -o pipefail
O=$PWD/gpurun_out/r05at; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py tests/test_gpu_fp8_encoder.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "attn or mx or fp8" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  echo "== attn old $i"; timeout -k 10 120 python -u scripts/attn_bench.py --lib scripts/exp/libtwhip_pre_attnvt.so 32 || exit $?
  echo "== attn new $i"; timeout -k 10 120 python -u scripts/attn_bench.py 32 || exit $?
done > $O/attn.txt 2>&1 || { tail -20 $O/attn.txt; exit 1; }
grep -v amdgpu.ids $O/attn.txt
for i in 1 2; do
  echo "== mx old $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000 --lib scripts/exp/libtwhip_pre_gelumx.so || exit $?
  echo "== mx new $i"; timeout -k 10 300 python -u scripts/gemm_mx_ab.py --variants 8 --m 96000 || exit $?
done > $O/mx.txt 2>&1 || { tail -20 $O/mx.txt; exit 1; }
grep -v amdgpu.ids $O/mx.txt
for c in c2 c5; do
  timeout -k 10 600 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  grep '^{' $O/$c.log | tail -1 > $O/$c.json
  python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['parity'], d['roofline']['achieved'], d['roofline']['frac'])"
done
