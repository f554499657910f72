# A/B of two in-tree builds on the bench: bash scripts/exp/ab_lib.sh libA.so libB.so [reps]
set -e
reps=${3:-2}
for i in $(seq 1 $reps); do
  for lib in "$1" "$2"; do
    TW_LIB=$PWD/turbo-whisper-workspace_amd/twamd/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.log 2>&1
    echo "$lib $(tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])")"
  done
done
