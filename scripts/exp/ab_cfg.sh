#!/bin/bash
# A/B of engine knobs on a chosen bench config: CFG=c3 bash scripts/exp/ab_cfg.sh "TAG1 VAR=VAL ..." ...
set -u
CFG=${CFG:-c2}
mkdir -p gpurun_out/ab
for spec in "$@"; do
  set -- $spec; tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab/$tag.log 2>&1 \
    || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab/$tag.log') if l.startswith('{')][-1]); print('$tag', d['ms_per_step'], d['value'], d['roofline']['achieved'])"
done
