# GEMV change check: parity tests, alone per-launch costs, in-situ decode breakdown, bench A/B of the K-slice cap
set -e
mkdir -p gpurun_out/gr
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemv or gemm_partial or skinny" -p no:cacheprovider > gpurun_out/gr/t.log 2>&1 || { tail -20 gpurun_out/gr/t.log; exit 1; }
tail -1 gpurun_out/gr/t.log
timeout -k 10 200 python scripts/gemv_bench.py --kws 0,4 > gpurun_out/gr/gv.log 2>&1
grep -v "serial_tail=1\|amdgpu" gpurun_out/gr/gv.log | head -14
timeout -k 10 200 python scripts/exp/insitu_breakdown.py --variant 1 > gpurun_out/gr/isb.log 2>&1
grep -v amdgpu gpurun_out/gr/isb.log
TW_GEMV_MAX_KW=4 timeout -k 10 200 python scripts/exp/insitu_breakdown.py --variant 1 > gpurun_out/gr/isb4.log 2>&1
grep -v amdgpu gpurun_out/gr/isb4.log
bash scripts/exp/ab_env.sh "TW_GEMV_MAX_KW=8" "TW_GEMV_MAX_KW=4" 2
