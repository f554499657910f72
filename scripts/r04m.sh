set -o pipefail
# round-4 final evidence, call 1: the whole GPU suite + config 2 (rocprof kernel stats, PMC traffic / MFMA, bench),
# then config 3 (full hour and one 8-GPU rank's share) and the as-shipped call
bash scripts/gpu_round.sh r04m || exit $?
O=gpurun_out/r04m
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_full.log 2>&1 || exit $?
grep '^{' $O/c3_full.log | tail -1 > profiles/r04m_c3_full.json
timeout -k 10 600 python -u bench.py --config c3 --c3-share 8 --steps 5 --warmup 2 --no-cpu-baseline > $O/c3_share8.log 2>&1 || exit $?
grep '^{' $O/c3_share8.log | tail -1 > profiles/r04m_c3_share8.json
timeout -k 10 600 python -u scripts/exp/as_shipped_rtf.py > $O/as_shipped.log 2>&1 || exit $?
tail -1 $O/as_shipped.log > profiles/r04m_as_shipped_beam5.json
echo final-c2-done
