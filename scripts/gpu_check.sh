set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider > gpurun_out/kern.log 2>&1; rc=$?
echo "kern rc=$rc"; tail -40 gpurun_out/kern.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu_e2e.py -q -m gpu -p no:cacheprovider > gpurun_out/e2e.log 2>&1; rc=$?
  echo "e2e rc=$rc"; tail -40 gpurun_out/e2e.log
fi
if [ $rc -le 1 ]; then
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
fi
