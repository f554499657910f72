set -o pipefail
# round-4 final evidence, call 3: config 3 (the full hour and one 8-GPU rank's share), the as-shipped call, then
# config 5's kernel stats / traffic / bench (tests ran in r04m)
O=gpurun_out/r04o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_full.log 2>&1 || exit $?
grep '^{' $O/c3_full.log | tail -1 > $O/c3_full.json
timeout -k 10 600 python -u bench.py --config c3 --c3-share 8 --steps 5 --warmup 2 --no-cpu-baseline > $O/c3_share8.log 2>&1 || exit $?
grep '^{' $O/c3_share8.log | tail -1 > $O/c3_share8.json
timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped.log 2>&1 || exit $?
tail -1 $O/as_shipped.log > $O/as_shipped_beam5.json
timeout -k 10 300 python -u scripts/vorbis_speed.py > $O/vorbis_speed.log 2>&1 || exit $?
cat $O/vorbis_speed.log
BENCH_ARGS="--config c5" bash scripts/gpu_round.sh r04o_c5 1 || exit $?
echo final-c3-c5-done
