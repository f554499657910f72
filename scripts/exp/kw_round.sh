# decoder GEMV K-slices per column group beside an encoder GEMM (insitu_breakdown, fc1-shaped GEMM storm)
set -e
mkdir -p gpurun_out/kw
for v in 1 65537 131073 262145; do
  timeout -k 10 200 python scripts/exp/insitu_breakdown.py --variant $v --epi 1 > gpurun_out/kw/isb_$v.log 2>&1
  echo "== $v"; grep -E "step:|gemv" gpurun_out/kw/isb_$v.log
done
