#!/bin/bash
# The drop-in called as the reference calls it (scripts/as_shipped_rtf.py): turbo and large-v3 on 10 minutes,
# and a 2-minute upload with and without the fused decoder launch. usage: bash scripts/gpu_as_shipped.sh TAG
set -u
TAG=${1:-r06q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run NAME ARGS...
  local name=$1; shift
  timeout -k 10 500 python -u scripts/as_shipped_rtf.py "$@" > $OUT/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $OUT/$name.log; exit 1; }
  grep '^{' $OUT/$name.log
}
run turbo10 --model large-v3-turbo --minutes 10
run turbo2 --model large-v3-turbo --minutes 2
run turbo2_fused --model large-v3-turbo --minutes 2 --fused 1
run largev3_10 --model large-v3 --minutes 10
