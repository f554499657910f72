#!/bin/bash
# One GPU-box session: parity tests, the bench line, a rocprofv3 kernel-trace summary, the two
# PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic and one for MFMA utilisation. Every GPU step has its own time limit and the
# chain stops at the first failure.  usage: [BENCH_ARGS="--config c5"] bash scripts/gpu_round.sh TAG [skip_tests]
# (a config-5 TAG must contain "_c5": bench.py reads profiles/*_c5_traffic.json for it)
set -u
TAG=${1:-r01}
SKIP_TESTS=${2:-0}
BA=${BENCH_ARGS:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] $name" 
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -4 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then echo "STOP after $name"; exit $rc; fi
}
if [ "$SKIP_TESTS" != "1" ]; then
  step tests 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread
  cp $OUT/tests.log profiles/${TAG}_gputest.txt
fi
step prof_kt 600 rocprofv3 --kernel-trace --stats -T -d $OUT/kt -o kt --output-format csv -- python bench.py $BA --profile-only --steps 2 --warmup 1
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o pmc --output-format csv -- python bench.py $BA --profile-only --steps 1 --warmup 0
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o pmc --output-format csv -- python bench.py $BA --profile-only --steps 1 --warmup 0
step pmc_mfma 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 -T -d $OUT/pmc_mfma -o pmc --output-format csv -- python bench.py $BA --profile-only --steps 1 --warmup 0
python scripts/summarize_prof.py $OUT > $OUT/summary.txt 2>&1
cp $OUT/traffic.json profiles/${TAG}_traffic.json   # bench.py reads the newest profiles/*traffic.json
[ -f $OUT/mfma.json ] && cp $OUT/mfma.json profiles/${TAG}_mfma.json
step bench 900 python bench.py $BA --steps 20 --warmup 5
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
cp $OUT/bench.json profiles/${TAG}_bench.json; cp $OUT/summary.txt profiles/${TAG}_rocprof_summary.txt
echo done
