# cross-attention load-unroll variants: in-situ breakdown beside an encoder GEMM, then the bench A/B
set -e
mkdir -p gpurun_out/cx
for v in 10 0x200000A; do
  TW_ATTN_VARIANT=$v timeout -k 10 200 python scripts/exp/insitu_breakdown.py --variant 1 --epi 1 > gpurun_out/cx/isb_$v.log 2>&1
  echo "== $v"; grep -E "step:|cross" gpurun_out/cx/isb_$v.log
done
bash scripts/exp/ab_multi.sh 2 10 TW_ATTN_VARIANT=10 TW_ATTN_VARIANT=0x200000A
