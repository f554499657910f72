set -o pipefail
# round-4 final evidence, call 2: config 3 (the full hour and one 8-GPU rank's share), the as-shipped call, then
# config 5's kernel stats / traffic / bench (tests ran in call 1)
O=gpurun_out/r04n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_full.log 2>&1 || exit $?
grep '^{' $O/c3_full.log | tail -1 > $O/c3_full.json
timeout -k 10 600 python -u bench.py --config c3 --c3-share 8 --steps 5 --warmup 2 --no-cpu-baseline > $O/c3_share8.log 2>&1 || exit $?
grep '^{' $O/c3_share8.log | tail -1 > $O/c3_share8.json
timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped.log 2>&1 || exit $?
tail -1 $O/as_shipped.log > $O/as_shipped_beam5.json
for kw in 1 4; do  # proj_out K-slices for decode passes alone: 1 vs 4 (the shipped default)
  TW_DEC_ALONE_WIDE_KW=$kw timeout -k 10 600 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/dec_kw$kw.log 2>&1 || exit $?
done
for dk in 0 1; do  # kernel arguments in device memory (HIP_FORCE_DEV_KERNARG): the decode step's per-launch floor
  HIP_FORCE_DEV_KERNARG=$dk timeout -k 10 600 python -u scripts/decode_step_time.py --rows 15 24 64 > $O/dec_devkernarg$dk.log 2>&1 || exit $?
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_devkernarg1.log 2>&1 || exit $?
grep '^{' $O/bench_devkernarg1.log | tail -1
TW_DEC_ALONE_WIDE_KW=1 timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped_kw1.log 2>&1 || exit $?
BENCH_ARGS="--config c5" bash scripts/gpu_round.sh r04n_c5 1 || exit $?
echo final-c3-c5-done
