#!/bin/bash
# The whole -m gpu suite (one process), log under gpurun_out/TAG. usage: bash scripts/gpu_tests.sh TAG
set -u
TAG=${1:-r06p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
exit $rc
