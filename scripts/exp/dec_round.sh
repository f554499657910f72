# decoder-kernel change check: full GPU suite, in-situ breakdown, bench line
set -e
mkdir -p gpurun_out/dr
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/dr/t.log 2>&1 || { grep -B5 -A30 "Error\|FAILED" gpurun_out/dr/t.log | head -60; exit 1; }
tail -1 gpurun_out/dr/t.log
timeout -k 10 200 python scripts/exp/insitu_breakdown.py --variant 1 > gpurun_out/dr/isb.log 2>&1
grep -v amdgpu gpurun_out/dr/isb.log
bash scripts/exp/env_sweep.sh "TW_ATTN_VARIANT=0x800" "TW_X=1" "TW_ATTN_VARIANT=0x800" "TW_X=1"
