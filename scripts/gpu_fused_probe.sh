#!/bin/bash
# tw_dec_fused per-phase timestamps (scripts/fused_probe.py) at 15 and 24 rows. usage: bash scripts/gpu_fused_probe.sh TAG
set -u
TAG=${1:-r06e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for R in 15 24; do
  timeout -k 10 300 python -u scripts/fused_probe.py --rows $R --pos 64 > $OUT/probe$R.log 2>&1 || exit $?
  head -2 $OUT/probe$R.log | tail -1
done
