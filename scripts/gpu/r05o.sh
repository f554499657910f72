set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_torch_ops.py tests/test_gpu_turbo.py tests/test_gpu_e2e.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 1; }
tail -2 $O/t.txt
bash scripts/gpu/ab_env20.sh TW_ENC_OPS=0 TW_ENC_OPS=1 3
