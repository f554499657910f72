set -e
for r in 0 4 6 8 10; do
  echo "== TW_DEC_CUS=$r"
  TW_DEC_CUS=$r timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cus_$r.log 2>&1
  tail -1 gpurun_out/cus_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
