#!/bin/bash
# decode pass alone per step, launch chain vs tw_dec_fused, at small row counts. usage: bash scripts/gpu_fused_rows.sh TAG
set -u
TAG=${1:-r06o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/decode_step_time.py --rows 1 2 4 8 12 --fused 0 1 --reps 3 > $OUT/step_time_small.log 2>&1
rc=$?
grep '^{' $OUT/step_time_small.log | grep step_us
exit $rc
