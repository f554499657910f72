#!/bin/bash
# One GPU-box pass: the GPU test suite (log kept for profiles/), smoke(), and one bench line. Each GPU step has its
# own time limit; a test FAILURE (pytest rc 1) still lets smoke/bench run, anything else (fault, abort, timeout)
# stops the chain.   usage: bash scripts/gpu_check.sh TAG [pytest selection...]
set -u
TAG=${1:-r03x}
shift || true
SEL=${*:-tests}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] tests: $SEL"
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rA \
  > $OUT/${TAG}_gputest.txt 2>&1
rc=$?
echo "[$(date +%T)] tests rc=$rc"; tail -3 $OUT/${TAG}_gputest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after tests"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.txt 2>&1
rc2=$?
echo "[$(date +%T)] smoke rc=$rc2"; tail -2 $OUT/${TAG}_smoke.txt
if [ $rc2 -ne 0 ]; then echo "STOP after smoke"; exit $rc2; fi
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > $OUT/${TAG}_bench.txt 2>&1
rc3=$?
echo "[$(date +%T)] bench rc=$rc3"; grep '^{' $OUT/${TAG}_bench.txt | tail -1 | cut -c1-600
exit $(( rc != 0 ? rc : rc3 ))
