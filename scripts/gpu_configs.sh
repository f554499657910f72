#!/bin/bash
# Config 3 (the hour on one GPU, and one rank's 8-way share) and config 5 (MX fp8 encoder, 64 windows) bench lines at
# HEAD, each step under its own time limit; the chain stops at the first failure.  usage: bash scripts/gpu_configs.sh TAG
set -u
TAG=${1:-r06c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; grep '^{' $OUT/$name.log | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
  grep '^{' $OUT/$name.log | tail -1 > $OUT/$name.json
}
step c3_full 900 python -u bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline
step c3_share8 900 python -u bench.py --config c3 --c3-share 8 --steps 10 --warmup 3 --no-cpu-baseline
step c5 900 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline
echo done
