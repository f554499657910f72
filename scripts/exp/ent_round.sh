# non-temporal GEMM epilogue stores (GB_EPI_NT build): decoder in situ beside k_gemm_big, then the bench A/B
set -e
mkdir -p gpurun_out/ent
for lib in libtwhip.so libtwhip_ent.so; do
  TW_LIB=turbo-whisper-workspace_amd/twamd/$lib timeout -k 10 200 python scripts/exp/insitu_breakdown.py --variant 1 --epi 1 > gpurun_out/ent/isb_$lib.log 2>&1
  echo "== $lib"; grep -v amdgpu gpurun_out/ent/isb_$lib.log | tail -7
done
bash scripts/exp/ab_multi.sh 2 10 - TW_LIB=turbo-whisper-workspace_amd/twamd/libtwhip_ent.so
