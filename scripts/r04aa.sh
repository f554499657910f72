set -o pipefail
# proj_out K-slices for decode steps beside an encoder chunk (the pipelined steady state): 1 (default) vs 2 vs 4
O=gpurun_out/r04aa; mkdir -p $O
export TMPDIR=/tmp
b() {  # b NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$name.log 2>&1 || exit $?
  echo "$name $(grep '^{' $O/bench_$name.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["parity"])')"
}
for r in 1 2 3; do
  b kw1_$r TW_DEC_BESIDE_WIDE_KW=1
  b kw2_$r TW_DEC_BESIDE_WIDE_KW=2
  b kw4_$r TW_DEC_BESIDE_WIDE_KW=4
done
echo sweep-done
