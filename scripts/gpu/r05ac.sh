# encoder store cache policy A/B on the 20-step bench: the shipped TW_ENC_NT (GEMM bf16 / GELU / other outputs
# non-temporal) vs every encoder store non-temporal (127) vs none (0); the library swapped in place between runs
set -o pipefail
O=gpurun_out/r05ac; mkdir -p $O
L=turbo-whisper-workspace_amd/twamd/libtwhip.so
cp $L $O/libtwhip_default.so
run() {
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit $?
  echo "$1 $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['parity'])")"
}
for i in 1 2; do
  cp $O/libtwhip_default.so $L; run default
  cp scripts/exp/libtwhip_ntall.so $L; run nt_all
  cp scripts/exp/libtwhip_ntnone.so $L; run nt_none
done
cp $O/libtwhip_default.so $L
