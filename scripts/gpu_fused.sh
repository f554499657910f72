#!/bin/bash
# tw_dec_fused on the GPU: its parity tests against the launch chain, then the decode pass alone per step with and
# without it. usage: bash scripts/gpu_fused.sh TAG [rows...]
set -u
TAG=${1:-r06d}
shift || true
ROWS=${*:-15 24}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] fused tests"
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_fused.py \
  > $OUT/fused_tests.log 2>&1
rc=$?
echo "[$(date +%T)] fused tests rc=$rc"; tail -5 $OUT/fused_tests.log
[ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] decode step time"
timeout -k 10 600 python -u scripts/decode_step_time.py --rows $ROWS --fused 0 1 --reps 3 > $OUT/step_time.log 2>&1
rc=$?
echo "[$(date +%T)] step time rc=$rc"; grep '^{' $OUT/step_time.log
exit $rc
