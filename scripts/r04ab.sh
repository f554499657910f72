set -o pipefail
# the pipelined step's balance on round-4 kernels (no profiler: HIP events on both streams), and bench.py as the driver
# runs it after the roofline field change
O=gpurun_out/r04ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/exp/timeline_events.py --steps 4 > $O/timeline.log 2>&1 || { tail -30 $O/timeline.log; exit 1; }
tail -25 $O/timeline.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline_decode"])'
