set -o pipefail
# encoder LayerNorm LDS request beside a decode (KiB): 0 (no cap) vs 34 / 40 / 48, interleaved config 2 bench
O=gpurun_out/r04y; mkdir -p $O
export TMPDIR=/tmp
b() {  # b NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$name.log 2>&1 || exit $?
  echo "$name $(grep '^{' $O/bench_$name.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["parity"])')"
}
for r in 1 2; do
  b ln0_$r TW_LN_PAD_BESIDE=0
  b ln34_$r TW_LN_PAD_BESIDE=34
  b ln40_$r TW_LN_PAD_BESIDE=40
  b ln48_$r TW_LN_PAD_BESIDE=48
done
echo sweep-done
