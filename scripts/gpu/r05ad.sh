# in-situ cost of a decoder launch: the fused select + next-step embedding (47 launches per token) against the two
# separate launches (49), 20-step bench, three interleaved pairs
set -o pipefail
O=gpurun_out/r05ad; mkdir -p $O
for i in 1 2 3; do
for e in "TW_PATCH=fused_select=1" "TW_PATCH=fused_select=0"; do
  env $e timeout -k 10 300 python -u scripts/exp/bench_patched.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit $?
  echo "$e $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
done
done
