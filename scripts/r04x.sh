set -o pipefail
# pipeline knob sweep on round-4 kernels (config 2 bench, interleaved): decode queue depth, encoder chunks ahead,
# encoder-attention LDS padding beside a decode (units of 16 KiB)
O=gpurun_out/r04x; mkdir -p $O
export TMPDIR=/tmp
b() {  # b NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$name.log 2>&1 || exit $?
  echo "$name $(grep '^{' $O/bench_$name.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["parity"])')"
}
for r in 1 2; do
  b base_$r TW_AB=0
  b dec2_$r TW_DEC_AHEAD=2
  b pump1_$r TW_PUMP_AHEAD=1
  b pump3_$r TW_PUMP_AHEAD=3
  b pad2_$r TW_ATTN_PAD_BESIDE=2
  b pad6_$r TW_ATTN_PAD_BESIDE=6
done
echo sweep-done
