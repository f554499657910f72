set -o pipefail
# combined call options + the wide proj_out K-slices (tests, then alone-decode / as-shipped A/B: 1 vs 4 slices)
O=gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_combos.py tests/test_gpu_word.py tests/test_gpu_longform.py tests/test_gpu_fallback.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|exact|differs|same transcript" $O/tests.log | tail -60
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemv" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gemv.log 2>&1 || { tail -30 $O/gemv.log; exit 1; }
tail -1 $O/gemv.log
for kw in 1 4; do
  TW_DEC_ALONE_WIDE_KW=$kw timeout -k 10 600 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/dec_kw$kw.log 2>&1 || exit $?
  echo "kw=$kw"; grep '^{' $O/dec_kw$kw.log
done
for kw in 1 4; do
  TW_DEC_ALONE_WIDE_KW=$kw timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped_kw$kw.log 2>&1 || exit $?
  echo "kw=$kw"; tail -1 $O/as_shipped_kw$kw.log
done
