set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_torch_ops.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/ops.txt 2>&1 || { tail -40 $O/ops.txt; exit 1; }
tail -3 $O/ops.txt
bash scripts/gpu/ab_env20.sh TW_ENC_OPS=0 TW_ENC_OPS=1 2
