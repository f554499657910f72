#!/bin/bash
# A/B (not product code): key-split count of the beam-grouped cross attention (DA_XSPLIT, build-time), as-shipped
# beam-5 call; rebuilds the library in this (scratch) tree for each value.
set -e
for ns in 3 6 2 4; do
  touch turbo-whisper-workspace_amd/csrc/attention.hip
  make -s -C turbo-whisper-workspace_amd/csrc -j16 EXTRA=-DDA_XSPLIT=$ns > /dev/null
  timeout -k 10 200 python -u scripts/exp/as_shipped_rtf.py > gpurun_out/xs_$ns.log 2>&1
  echo "DA_XSPLIT=$ns: $(tail -1 gpurun_out/xs_$ns.log)"
done
