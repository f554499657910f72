#!/bin/bash
# A/B of engine knobs on the default bench (config 2), one bench process per setting:
#   bash scripts/ab_bench.sh "TAG1 VAR=VAL ..." "TAG2 VAR=VAL ..." ...
set -u
mkdir -p gpurun_out/ab
for spec in "$@"; do
  set -- $spec; tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab/$tag.log 2>&1 \
    || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/$tag.log') if l.startswith('{')][-1]); print('$tag', d['ms_per_step'], d['value'], d['roofline']['achieved'])"
done
