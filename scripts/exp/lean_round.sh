# decoder co-residency beside the 8-phase encoder GEMM: per-kernel in-situ costs (default build vs the
# TW_DEC_WPE=6 build) beside k_gemm_big (1) and k_gemm_8p (5)
set -e
mkdir -p gpurun_out/lean
for lib in libtwhip.so libtwhip_lean.so; do
  for v in 1 5; do
    TW_LIB=turbo-whisper-workspace_amd/twamd/$lib timeout -k 10 200 python scripts/exp/insitu_breakdown.py --variant $v --epi 1 > gpurun_out/lean/isb_${lib}_$v.log 2>&1
    echo "== $lib gemm variant $v"; grep -v amdgpu gpurun_out/lean/isb_${lib}_$v.log | tail -7
  done
done
