#!/bin/bash
# MX fp8 bring-up: the lane-map probe, then the MX kernel and config-5 end-to-end tests.
set -u
mkdir -p gpurun_out/mx
timeout -k 10 60 ./scripts/exp/mx_probe > gpurun_out/mx/probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/mx/probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8_encoder.py -x -v -s --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/mx/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/mx/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_bench.py --rounds 3 > gpurun_out/mx/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; cat gpurun_out/mx/gemm_bench.log
exit $rc
