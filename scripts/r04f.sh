set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/beam -o kt --output-format csv -- python -u scripts/exp/beam_prof.py > $O/beam.log 2>&1 || exit $?
tail -3 $O/beam.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/dec -o kt --output-format csv -- python -u scripts/decode_step_time.py --rows 24 --reps 1 > $O/dec.log 2>&1 || exit $?
tail -2 $O/dec.log
